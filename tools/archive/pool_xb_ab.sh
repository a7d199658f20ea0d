#!/bin/bash
# S3D with maxpool3_s1 (FAC_POOL_XB=1) vs maxpool3_s1x at 2 / 4 output columns per thread, same box, twice.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
for xb in 1 2 4; do
  FAC_POOL_XB=$xb timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -q --timeout 200 --timeout-method thread -k "pool or s3d" > gpurun_out/poolxb_tests_$xb.log 2>&1 || { tail -20 gpurun_out/poolxb_tests_$xb.log; exit 1; }
  echo "xb=$xb $(tail -1 gpurun_out/poolxb_tests_$xb.log)"
done
for rep in 1 2; do for xb in 1 2 4; do
  FAC_POOL_XB=$xb timeout -k 10 200 python -u bench.py --only s3d --steps 10 --warmup 3 > gpurun_out/poolxb_$xb.log 2>&1 || { tail -5 gpurun_out/poolxb_$xb.log; exit 1; }
  python -c "import json; l=json.loads(open('gpurun_out/poolxb_$xb.log').read().strip().splitlines()[-1]); print('xb=$xb', l['value'], l['ms_per_step'])"
done; done
