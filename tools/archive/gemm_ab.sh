#!/bin/bash
# GEMM tile variants: parity, isolated sweep, then pipelined-bench A/B arms.
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -m gpu -x --timeout 120 --timeout-method thread \
  -k "gemm_variants or b256 or native_library" > gpurun_out/gemm_test.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/gemm_test.log; exit 1; }
tail -1 gpurun_out/gemm_test.log
timeout -k 10 300 python tools/gemm_sweep.py > gpurun_out/gemm_sweep.log 2>&1 || { tail -5 gpurun_out/gemm_sweep.log; exit 1; }
bash tools/ab_bench.sh "$@"
