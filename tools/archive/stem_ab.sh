#!/bin/bash
# Stem kernel change: parity subset, then same-box A/B against libfac_cvit_base.so,
# then option arms ($AB_ARMS, ';'-separated bench flag sets) on the tree build.
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -m gpu -x --timeout 120 --timeout-method thread \
  -k "fused_stem224 or c1_single or b256 or pipelined or native_library or chunking or graph" > gpurun_out/ab_test.log 2>&1 || { echo "tests failed"; tail -20 gpurun_out/ab_test.log; exit 1; }
tail -2 gpurun_out/ab_test.log
bash tools/ab_lib.sh "$@" || exit 1
if [ -n "$AB_ARMS" ]; then
  IFS=';' read -ra A <<< "$AB_ARMS"
  bash tools/ab_bench.sh "${A[@]}"
fi
