#!/bin/bash
# Round-4 evidence pass on one GPU box: every GPU test, the default bench
# line, then kernel traces + PMC passes of configs 4/5 (tools/profile_cfg45_r03.sh,
# tools/pmc_cfg45_r03.sh with PROF_TAG=r04).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -rA > gpurun_out/pytest_gpu.log 2>&1 || { grep -E "FAILED|Error" gpurun_out/pytest_gpu.log | head -20; tail -5 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -5 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 600 python -u bench.py > gpurun_out/bench.log 2>&1 || { tail -5 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log | cut -c1-300
[ -n "$NO_PROF" ] && exit 0
PROF_TAG=r04 bash tools/profile_cfg45_r03.sh || exit 1
PROF_TAG=r04 bash tools/pmc_cfg45_r03.sh || exit 1
