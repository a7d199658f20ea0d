#!/bin/bash
# Round 6: deferred encoder -- HEAD vs the previous lib (4 alternations) and
# the encoder stream's priority with the deferral.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
PREV=ab/libfac_cvit_predefer.so DTYPES="bf16 fp16" REPS=4 STEPS=60 bash tools/lib_ab_cvit.sh || exit 1
ARMS="tail_priority=1;tail_priority=0" REPS=2 DTYPES="bf16 fp16" STEPS=60 bash tools/ab_bench.sh
