#!/bin/bash
# Round 6, first box: vendor-GEMM ceiling for the conv shapes, per-layer conv
# times at B = 256 (both dtypes), and the default bench line at HEAD.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/gemm_ceiling.py > gpurun_out/gemm_ceiling.txt 2>&1 || { tail -5 gpurun_out/gemm_ceiling.txt; exit 1; }
tail -1 gpurun_out/gemm_ceiling.txt | cut -c1-200
for dt in fp16 bf16; do
  timeout -k 10 200 python -u tools/conv_sweep.py --dtype $dt --tag $dt > gpurun_out/sweep_$dt.txt 2>&1 || { tail -5 gpurun_out/sweep_$dt.txt; exit 1; }
  tail -1 gpurun_out/sweep_$dt.txt
done
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_base.log 2>&1 || { tail -5 gpurun_out/bench_base.log; exit 1; }
tail -1 gpurun_out/bench_base.log | cut -c1-400
