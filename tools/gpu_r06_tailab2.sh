#!/bin/bash
# Round 6: tail GEMM tile variants in the pipelined headline, second pass
# (more arms and alternations).
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
ARMS="gemm_qkv=-1;gemm_qkv=0 gemm_out=0 gemm_ff1=0 gemm_ff2=0 gemm_head=0;gemm_qkv=1 gemm_out=1 gemm_ff1=1 gemm_ff2=1 gemm_head=1;gemm_qkv=0 gemm_ff1=0 gemm_head=0;gemm_out=0 gemm_ff2=0" REPS=3 DTYPES="fp16 bf16" STEPS=40 bash tools/ab_bench.sh
