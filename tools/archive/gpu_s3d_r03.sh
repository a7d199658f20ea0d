#!/bin/bash
# S3D per-block parity tests, then config 4/5 throughput at larger batches.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_ops.py -x -q --timeout 300 --timeout-method thread -k "s3d" -rA > gpurun_out/r03_s3d_tests.log 2>&1 || { tail -30 gpurun_out/r03_s3d_tests.log; exit 1; }
tail -1 gpurun_out/r03_s3d_tests.log
for b in ${S3D_BS:-384 512}; do
  timeout -k 10 200 python -u bench.py --only s3d --s3d-batch $b --steps 10 --warmup 3 > gpurun_out/r03_bs_s3d_$b.log 2>&1 || { tail -5 gpurun_out/r03_bs_s3d_$b.log; exit 1; }
  python -c "import json; l=json.loads(open('gpurun_out/r03_bs_s3d_$b.log').read().strip().splitlines()[-1]); print('s3d B=$b', l['value'], l['ms_per_step'], l['conv_pool_layer_roofline']['fraction_of_step'])"
done
for b in ${RVK_BS:-768 1024}; do
  timeout -k 10 200 python -u bench.py --only resvitkan --rvk-batch $b --steps 10 --warmup 3 > gpurun_out/r03_bs_rvk_$b.log 2>&1 || { tail -5 gpurun_out/r03_bs_rvk_$b.log; exit 1; }
  python -c "import json; l=json.loads(open('gpurun_out/r03_bs_rvk_$b.log').read().strip().splitlines()[-1]); print('rvk B=$b', l['value'], l['ms_per_step'], l['conv_pool_layer_roofline']['fraction_of_step'])"
done
