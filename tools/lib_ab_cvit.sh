#!/bin/bash
# Same-box A/B of the in-tree library against a previous build (PREV, via
# FAC_CVIT_LIB) on the headline CViT line: value, stem launch and stage_ms.
#   PREV=ab/libfac_cvit_head.so DTYPES="bf16 fp16" REPS=3 TESTK=expr bash tools/lib_ab_cvit.sh
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
if [ -n "$TESTK" ]; then
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "$TESTK" > gpurun_out/labc_pytest.log 2>&1 || { tail -30 gpurun_out/labc_pytest.log; exit 1; }
  tail -1 gpurun_out/labc_pytest.log
fi
ARGS="--steps ${STEPS:-30} --warmup 5 --no-cpu-baseline --no-fp16-line --no-video --no-s3d --no-resvitkan --no-repbn8"
for rep in $(seq 1 ${REPS:-3}); do
  for arm in prev cur; do
    for dt in ${DTYPES:-bf16}; do
      if [ $arm = prev ]; then export FAC_CVIT_LIB=$PREV; else unset FAC_CVIT_LIB; fi
      timeout -k 10 120 python -u bench.py $ARGS --dtype $dt > gpurun_out/labc_${arm}_${dt}_$rep.log 2>&1 || { tail -5 gpurun_out/labc_${arm}_${dt}_$rep.log; exit 1; }
      python - gpurun_out/labc_${arm}_${dt}_$rep.log $arm $dt <<'PY'
import json,sys
l=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); s=l['stage_ms']
print('%-4s %-5s %9.1f stem_launch %.4f ' % (sys.argv[2], sys.argv[3], l['value'], l['roofline']['launch_ms']) + ' '.join('%s=%.4f' % (k[4:], s[k]) for k in s if k.startswith('conv') and k not in ('conv2', 'conv3')))
PY
    done
  done
done
unset FAC_CVIT_LIB
