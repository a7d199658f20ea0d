#!/bin/bash
# Round 5: few-crop + Winograd tests, the reference-mode latency breakdown,
# then the fp16 / bf16 CViT line with option wino = 0 / 1 / 3 / 7 (same box).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "${TESTK:-gemm or few_crop or graph or two_streams or out_of_range or batch or wino}" > gpurun_out/t.log 2>&1; rc=$?
tail -3 gpurun_out/t.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" gpurun_out/t.log | head -20; exit 1; }
if [ -z "$NO_LAT" ]; then
  timeout -k 10 240 python -u tools/ref_latency.py > gpurun_out/ref_latency.txt 2>&1 || exit 1
  cat gpurun_out/ref_latency.txt | grep -v amdgpu.ids
fi
ARGS="--steps 30 --warmup 5 --no-cpu-baseline --no-fp16-line --no-video --no-s3d --no-resvitkan --no-repbn8"
for rep in 1 2; do
for dt in fp16 bf16; do
for w in 0 1 3 7; do
  timeout -k 10 120 python -u bench.py $ARGS --dtype $dt --opt wino=$w > gpurun_out/wino_${dt}_${w}_$rep.log 2>&1 || exit 1
  python - gpurun_out/wino_${dt}_${w}_$rep.log $dt $w <<'PY'
import json,sys
l=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); s=l['stage_ms']
print(sys.argv[2], 'wino', sys.argv[3], 'value', l['value'], 'parity', l['parity']['max_abs_dprob'] if l['parity'] else None,
      'c7-9 %.3f c10-13 %.3f c14-17 %.3f' % (sum(s[f'conv{i}'] for i in (7,8,9)), sum(s[f'conv{i}'] for i in (10,11,12,13)), sum(s[f'conv{i}'] for i in (14,15,16,17))))
PY
done; done; done
