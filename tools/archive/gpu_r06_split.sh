#!/bin/bash
# Round 6: wave-specialised stem (option stem_split) -- parity, then A/B on the headline.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
ARMS="stem_split=0;stem_split=1" REPS=${REPS:-3} DTYPES="bf16 fp16" STEPS=40 TESTK="stem_split or fused_stem224 or graph_replay" bash tools/ab_bench.sh
