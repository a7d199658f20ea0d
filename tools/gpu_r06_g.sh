#!/bin/bash
# Round 6: 128x128 encoder GEMM tiles in the pipelined headline, same box.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -k "gemm_variants" > gpurun_out/g_pytest.log 2>&1 || { tail -20 gpurun_out/g_pytest.log; exit 1; }
tail -1 gpurun_out/g_pytest.log
ARMS="gemm_qkv=-1;gemm_qkv=7 gemm_out=7 gemm_ff1=7 gemm_ff2=7 gemm_head=7;gemm_qkv=7 gemm_ff1=7" REPS=3 DTYPES="fp16 bf16" STEPS=40 bash tools/ab_bench.sh
