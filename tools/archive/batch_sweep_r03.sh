#!/bin/bash
# Config 4/5 throughput vs batch per step (same box): S3D clips 64/128/256, ResVitKan crops 256/512.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
for b in 64 128 256; do
  timeout -k 10 200 python -u bench.py --only s3d --s3d-batch $b --steps 10 --warmup 3 > gpurun_out/r03_bs_s3d_$b.log 2>&1 || { tail -5 gpurun_out/r03_bs_s3d_$b.log; exit 1; }
  python -c "import json; l=json.loads(open('gpurun_out/r03_bs_s3d_$b.log').read().strip().splitlines()[-1]); print('s3d B=$b', l['value'], l['ms_per_step'], l['conv_pool_layer_roofline']['fraction_of_step'])"
done
for b in 256 512; do
  timeout -k 10 200 python -u bench.py --only resvitkan --rvk-batch $b --steps 10 --warmup 3 > gpurun_out/r03_bs_rvk_$b.log 2>&1 || { tail -5 gpurun_out/r03_bs_rvk_$b.log; exit 1; }
  python -c "import json; l=json.loads(open('gpurun_out/r03_bs_rvk_$b.log').read().strip().splitlines()[-1]); print('rvk B=$b', l['value'], l['ms_per_step'], l['conv_pool_layer_roofline']['fraction_of_step'])"
done
