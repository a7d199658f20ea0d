#!/bin/bash
# Round 6: per-layer event timings of configs 4/5 at the bench batches (tools/rvk_layers.py).
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/rvk_layers.py --model s3d --B 1536 --u8 --reps 3 > gpurun_out/r06_s3d_layers.txt 2>&1 || { tail -5 gpurun_out/r06_s3d_layers.txt; exit 1; }
tail -2 gpurun_out/r06_s3d_layers.txt
timeout -k 10 300 python -u tools/rvk_layers.py --model rvk --B 3072 --reps 3 > gpurun_out/r06_resvitkan_layers.txt 2>&1 || { tail -5 gpurun_out/r06_resvitkan_layers.txt; exit 1; }
tail -2 gpurun_out/r06_resvitkan_layers.txt
