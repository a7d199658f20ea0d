#!/bin/bash
# Round-4 evidence on one GPU box: every GPU test, then the default bench line.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -rA > gpurun_out/pytest_gpu.log 2>&1 || { grep -E "FAILED|Error|error" gpurun_out/pytest_gpu.log | head -20; tail -5 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
[ -n "$NO_BENCH" ] && exit 0
timeout -k 10 600 python -u bench.py > gpurun_out/bench.log 2>&1 || { tail -5 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log | cut -c1-400
