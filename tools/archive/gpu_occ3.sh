#!/bin/bash
# A/B: conv_occ3 arms (one halo buffer, 3 workgroups per CU) on the headline line
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
ARMS="conv_occ3=0;conv_occ3=1;conv_occ3=2;conv_occ3=4" DTYPES="bf16" REPS=2 TESTK="each_conv or b256_config2" bash tools/ab_bench.sh
