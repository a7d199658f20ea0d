#!/bin/bash
# Round 6: tail GEMM tile variants in the pipelined headline (LDS footprint of
# the co-running encoder GEMMs), same box, two alternations.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
ARMS="gemm_qkv=-1;gemm_qkv=6 gemm_out=6 gemm_ff1=6 gemm_ff2=6 gemm_head=6;gemm_qkv=4 gemm_out=4 gemm_ff1=4 gemm_ff2=4 gemm_head=4;gemm_qkv=0 gemm_out=0 gemm_ff1=0 gemm_ff2=0 gemm_head=0" REPS=2 DTYPES="bf16 fp16" bash tools/ab_bench.sh
