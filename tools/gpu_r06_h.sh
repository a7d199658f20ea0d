#!/bin/bash
# Round 6: deferred pipelined encoder (starts after the next batch's stem):
# pipeline/graph/ordering tests, then the headline against the previous lib.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "pipelined or video or graph or few_crop or weights_changed or golden or chunked" > gpurun_out/h_pytest.log 2>&1 || { grep -E "FAILED|Error|error" gpurun_out/h_pytest.log | head -20; tail -5 gpurun_out/h_pytest.log; exit 1; }
tail -1 gpurun_out/h_pytest.log
PREV=ab/libfac_cvit_predefer.so DTYPES="bf16 fp16" REPS=3 STEPS=40 bash tools/lib_ab_cvit.sh || exit 1
