#!/bin/bash
# Round 6: the pipelined encoder on a CU-masked tail stream (option tail_cus) -- A/B on the headline.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
ARMS="tail_cus=0;tail_cus=16;tail_cus=32;tail_cus=64" REPS=${REPS:-2} DTYPES="bf16 fp16" STEPS=40 TESTK="pipelined" bash tools/ab_bench.sh
