#!/bin/bash
# Round 6: 112^2 box order (option box_rev) A/B on the headline, then the
# conv6 FETCH/WRITE A/B of the round-4 tree against HEAD.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
ARMS="box_rev=0;box_rev=2;box_rev=4;box_rev=6" REPS=3 DTYPES="bf16" STEPS=40 TESTK="box_rev" bash tools/ab_bench.sh || exit 1
bash tools/gpu_r06_c6fetch.sh || exit 1
echo boxrev ok
