#!/bin/bash
# S3D GPU parity tests, per-layer timings (256 clips) and the config-4 bench line.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
T=${TAG:-x}
timeout -k 10 400 python -u -m pytest tests/test_gpu_ops.py -x -q --timeout 300 --timeout-method thread -k "s3d or conv_nd or conv_tk or split" > gpurun_out/s3dc_tests_$T.log 2>&1 || { tail -30 gpurun_out/s3dc_tests_$T.log; exit 1; }
tail -1 gpurun_out/s3dc_tests_$T.log
timeout -k 10 200 python3 -u tools/rvk_layers.py --model s3d --B 256 > gpurun_out/s3dc_layers_$T.txt 2>&1 || { tail -5 gpurun_out/s3dc_layers_$T.txt; exit 1; }
head -8 gpurun_out/s3dc_layers_$T.txt | tail -6; grep -E "3x1x1/11 (192|128)->" gpurun_out/s3dc_layers_$T.txt; tail -1 gpurun_out/s3dc_layers_$T.txt
timeout -k 10 200 python -u bench.py --only s3d --steps 10 --warmup 3 > gpurun_out/s3dc_bench_$T.log 2>&1 || { tail -5 gpurun_out/s3dc_bench_$T.log; exit 1; }
python -c "import json; l=json.loads(open('gpurun_out/s3dc_bench_$T.log').read().strip().splitlines()[-1]); print('s3d', l['value'], l['ms_per_step'], l['conv_pool_layer_roofline']['fraction_of_step'])"
