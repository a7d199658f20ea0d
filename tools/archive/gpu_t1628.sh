#!/bin/bash
# 16x28 boxes for the 112^2 layers: conv tests (per-layer oracle + the
# golden forwards) on the new library, then the CViT bench and the per-layer
# sweep for base / new / alt libraries, alternating.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "golden or each_conv or conv45 or b32" > gpurun_out/pytest_t1628.log 2>&1 || { grep -E "FAILED|Error|assert" gpurun_out/pytest_t1628.log | head -20; tail -3 gpurun_out/pytest_t1628.log; exit 1; }
tail -1 gpurun_out/pytest_t1628.log
ARGS="--steps 50 --warmup 10 --no-fp16-line --no-video --no-s3d --no-resvitkan --no-repbn8 --no-cpu-baseline"
for rep in 1 2 3; do for v in base new alt; do
  case $v in base) export FAC_CVIT_LIB=$R/fac_fake_amd/libfac_cvit_base.so;; alt) export FAC_CVIT_LIB=$R/fac_fake_amd/libfac_cvit_alt.so;; *) unset FAC_CVIT_LIB;; esac
  timeout -k 10 200 python -u bench.py $ARGS > gpurun_out/t1628_$v.log 2>&1 || { tail -5 gpurun_out/t1628_$v.log; exit 1; }
  python -c "import json; l=json.loads(open('gpurun_out/t1628_$v.log').read().strip().splitlines()[-1]); s=l['stage_ms']; print('$v', l['value'], l['ms_per_step'], s['conv4'], s['conv5'], s['conv6'])"
done; done
