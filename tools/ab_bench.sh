#!/bin/bash
# Same-box A/B of bench.py option arms on the headline CViT line (stage_ms of
# the 112^2..14^2 convs beside the throughput), alternating arms, REPS rounds.
#   ARMS="conv112_wr=0;conv112_wr=1" DTYPES="fp16 bf16" REPS=2 TESTK=expr bash tools/ab_bench.sh
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
if [ -n "$TESTK" ]; then
  timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -k "$TESTK" > gpurun_out/ab_pytest.log 2>&1 || { tail -30 gpurun_out/ab_pytest.log; exit 1; }
  tail -1 gpurun_out/ab_pytest.log
fi
ARGS="--steps ${STEPS:-30} --warmup 5 --no-cpu-baseline --no-fp16-line --no-video --no-s3d --no-resvitkan --no-repbn8"
IFS=';' read -ra AR <<< "$ARMS"
for rep in $(seq 1 ${REPS:-2}); do
for arm in "${AR[@]}"; do
for dt in ${DTYPES:-fp16 bf16}; do
  opts=""; for o in $arm; do opts="$opts --opt $o"; done
  tag=$(echo "$arm" | tr ' =' '__')
  timeout -k 10 120 python -u bench.py $ARGS --dtype $dt $opts > gpurun_out/ab_${dt}_${tag}_$rep.log 2>&1 || { tail -5 gpurun_out/ab_${dt}_${tag}_$rep.log; exit 1; }
  python - gpurun_out/ab_${dt}_${tag}_$rep.log $dt "$arm" <<'PY'
import json,sys
l=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); s=l['stage_ms']
print('%-5s %-28s %9.1f  ' % (sys.argv[2], sys.argv[3], l['value']) + ' '.join('%s=%.4f' % (k[4:], s[k]) for k in s if k.startswith('conv') and k not in ('conv2', 'conv3')))
PY
done; done; done
