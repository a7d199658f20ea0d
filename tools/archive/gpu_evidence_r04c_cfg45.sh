#!/bin/bash
# Round-4 evidence pass c, configs 4/5: kernel traces, per-layer timings and
# PMC passes (tools/profile_cfg45_r03.sh, tools/pmc_cfg45_r03.sh, PROF_TAG=r04c).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
PROF_TAG=r04c bash tools/profile_cfg45_r03.sh || exit 1
PROF_TAG=r04c bash tools/pmc_cfg45_r03.sh || exit 1
