#!/bin/bash
# S3D bench with maxpool3_s1 at 1 / 2 / 4 / 8 output frames per thread (FAC_POOL_ZG), same box, twice.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -q --timeout 200 --timeout-method thread -k "pool or s3d" > gpurun_out/pool_tests.log 2>&1 || { tail -20 gpurun_out/pool_tests.log; exit 1; }
tail -1 gpurun_out/pool_tests.log
for rep in 1 2; do for zg in 8 4 2 1; do
  FAC_POOL_ZG=$zg timeout -k 10 200 python -u bench.py --only s3d --steps 10 --warmup 3 > gpurun_out/pool_zg$zg.log 2>&1 || { tail -5 gpurun_out/pool_zg$zg.log; exit 1; }
  python -c "import json; l=json.loads(open('gpurun_out/pool_zg$zg.log').read().strip().splitlines()[-1]); print('zg=$zg', l['value'], l['ms_per_step'])"
done; done
