#!/bin/bash
# config 5 / config 4 per-GPU batch sweep with the round-3 persistent conv kernels
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
for b in 512 768 1024; do
  timeout -k 10 300 python -u bench.py --only resvitkan --rvk-batch $b --steps 10 --warmup 3 > gpurun_out/bs.log 2>&1 || { tail -5 gpurun_out/bs.log; exit 1; }
  python -c "import json; l=json.loads(open('gpurun_out/bs.log').read().strip().splitlines()[-1]); print('rvk B=$b', l['value'], l['ms_per_step'], l['conv_pool_layer_roofline']['fraction_of_step'])"
done
for b in 256 384; do
  timeout -k 10 300 python -u bench.py --only s3d --s3d-batch $b --steps 10 --warmup 3 > gpurun_out/bs.log 2>&1 || { tail -5 gpurun_out/bs.log; exit 1; }
  python -c "import json; l=json.loads(open('gpurun_out/bs.log').read().strip().splitlines()[-1]); print('s3d B=$b', l['value'], l['ms_per_step'], l['conv_pool_layer_roofline']['fraction_of_step'])"
done
