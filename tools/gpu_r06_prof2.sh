#!/bin/bash
# Round-6 second-session profile pass (tag b): the headline's kernel trace and
# PMC passes (tools/profile_r06.sh) and the configs-4/5 PMC passes
# (tools/pmc_cfg45.sh).  GPU box only; summarise with tools/rocprof_summary.py
# and tools/pmc_cfg45_summary.py.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
PROF_TAG=b bash tools/profile_r06.sh || exit 1
PROF_TAG=b bash tools/pmc_cfg45.sh || exit 1
echo prof ok
