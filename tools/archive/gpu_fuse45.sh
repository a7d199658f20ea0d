#!/bin/bash
# conv45_fused: bit-equality + golden tests, then the CViT bench against
# libfac_cvit_base.so, alternating.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "conv45 or golden or each_conv or fused_stem or pipelined" > gpurun_out/pytest_f45.log 2>&1 || { grep -E "FAILED|Error|assert" gpurun_out/pytest_f45.log | head -20; tail -3 gpurun_out/pytest_f45.log; exit 1; }
tail -1 gpurun_out/pytest_f45.log
REPS=${REPS:-3} bash tools/lib_ab.sh
