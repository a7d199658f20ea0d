#!/bin/bash
# round 5: few-crop 14^2 convs with the 9-slice weight ring (conv_ring9), B = 29 forward A/B
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -k "ring9 or each_conv_kernel or few_crop or graph_replay" > gpurun_out/d_pytest.log 2>&1 || { tail -30 gpurun_out/d_pytest.log; exit 1; }
tail -1 gpurun_out/d_pytest.log
for r in 1 2 3; do for v in 0 1; do
  timeout -k 10 120 python -u tools/small_b_trace.py --graph --opt conv_ring9=$v > gpurun_out/ring9_$v.log 2>&1 || { tail -5 gpurun_out/ring9_$v.log; exit 1; }
  echo "conv_ring9=$v $(tail -1 gpurun_out/ring9_$v.log)"
done; done
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 180 rocprofv3 --kernel-trace -d gpurun_out/prof_small9 -o small -- python tools/small_b_trace.py --graph --opt conv_ring9=1 > gpurun_out/prof_small9.log 2>&1 || { tail -5 gpurun_out/prof_small9.log; exit 1; }
tail -1 gpurun_out/prof_small9.log
