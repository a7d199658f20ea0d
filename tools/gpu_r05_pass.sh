#!/bin/bash
# Round-5 evidence pass: every GPU test, smoke, the default bench line, the
# 112^2 conv A/B arms (options conv112 / conv_persist, same box, alternating),
# the reference-mode latency breakdown, then the headline profile passes.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -rA > gpurun_out/pytest_gpu.log 2>&1 || { grep -E "FAILED|Error" gpurun_out/pytest_gpu.log | head -20; tail -5 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -5 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 600 python -u bench.py > gpurun_out/bench.log 2>&1 || { tail -5 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log | cut -c1-300
ARGS="--steps 30 --warmup 5 --no-cpu-baseline --no-fp16-line --no-video --no-s3d --no-resvitkan --no-repbn8"
for rep in 1 2; do
for arm in "conv112=0 --opt conv_persist=0" "conv112=0 --opt conv_persist=1" "conv112=1 --opt conv_persist=1" "conv112=2 --opt conv_persist=1"; do
for dt in fp16 bf16; do
  tag=$(echo "$arm" | tr -d ' -' | tr '=' '_')
  timeout -k 10 120 python -u bench.py $ARGS --dtype $dt --opt $arm > gpurun_out/ab_${dt}_${tag}_$rep.log 2>&1 || exit 1
  python - gpurun_out/ab_${dt}_${tag}_$rep.log $dt "$arm" <<'PY'
import json,sys
l=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); s=l['stage_ms']
print(sys.argv[2], sys.argv[3], 'value', l['value'], 'c4 %.4f c5 %.4f c6 %.4f' % (s['conv4'], s['conv5'], s['conv6']))
PY
done; done; done
timeout -k 10 240 python -u tools/ref_latency.py > gpurun_out/ref_latency.txt 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/ref_latency.txt
PROF_TAG=a bash tools/profile_r05.sh || exit 1
