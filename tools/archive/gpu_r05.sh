#!/bin/bash
# Round-5 evidence pass: every GPU test, smoke, the default bench line.
# NO_BENCH=1 skips the bench; NO_TESTS=1 skips the tests.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -rA > gpurun_out/pytest_gpu.log 2>&1 || { grep -E "FAILED|Error" gpurun_out/pytest_gpu.log | head -20; tail -5 gpurun_out/pytest_gpu.log; exit 1; }
  tail -1 gpurun_out/pytest_gpu.log
  timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -5 gpurun_out/smoke.log; exit 1; }
  tail -1 gpurun_out/smoke.log
fi
if [ -z "$NO_BENCH" ]; then
  timeout -k 10 600 python -u bench.py $BENCH_ARGS > gpurun_out/bench.log 2>&1 || { tail -5 gpurun_out/bench.log; exit 1; }
  tail -1 gpurun_out/bench.log | cut -c1-400
fi
