#!/bin/bash
# Round 6: stem_split orders (1 skewed, 2 conv3 first, 3 conv1 first) against the fused stem.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
ARMS="stem_split=0;stem_split=1;stem_split=2;stem_split=3" REPS=2 DTYPES="bf16" STEPS=40 TESTK="stem_split" bash tools/ab_bench.sh
