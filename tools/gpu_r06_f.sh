#!/bin/bash
# Round 6: split-K of the encoder's to_out / FF2 projections (proj_splits) and
# the tail stream priority in the pipelined headline, same box.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
ARMS="proj_splits=4;proj_splits=2;proj_splits=1;tail_priority=0" REPS=2 DTYPES="fp16 bf16" STEPS=40 bash tools/ab_bench.sh
