#!/bin/bash
# 28^2 split last round: the conv bit-equality tests, then per-layer sweep +
# CViT bench against libfac_cvit_base.so, alternating.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "conv_db or each_conv or golden" > gpurun_out/pytest_split.log 2>&1 || { grep -E "FAILED|Error|assert" gpurun_out/pytest_split.log | head -20; tail -3 gpurun_out/pytest_split.log; exit 1; }
tail -1 gpurun_out/pytest_split.log
LAYERS=9,10,11,12 REPS=3 bash tools/gpu_libab.sh
