#!/bin/bash
# Round-3 GPU-box evidence: every GPU test, the default bench line, smoke,
# then the config-2 profile passes (tools/profile_r03.sh).  TAG names the logs.
R=${GRAFT_REPO_ROOT:-$(pwd)}
T=${TAG:-a}
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -rA > gpurun_out/r03_pytest_$T.log 2>&1 || { tail -30 gpurun_out/r03_pytest_$T.log; exit 1; }
tail -1 gpurun_out/r03_pytest_$T.log
timeout -k 10 600 python -u bench.py > gpurun_out/r03_bench_$T.log 2>&1 || { tail -5 gpurun_out/r03_bench_$T.log; exit 1; }
tail -1 gpurun_out/r03_bench_$T.log | cut -c1-600
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03_smoke_$T.log 2>&1 || { tail -5 gpurun_out/r03_smoke_$T.log; exit 1; }
tail -1 gpurun_out/r03_smoke_$T.log
if [ -n "$PROFILE" ]; then
  bash tools/profile_r03.sh || exit $?
fi
