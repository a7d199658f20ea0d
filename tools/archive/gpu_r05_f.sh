#!/bin/bash
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -k "ring9 or graph or weights_changed or few_crop or each_conv" > gpurun_out/f_pytest.log 2>&1 || { tail -30 gpurun_out/f_pytest.log; exit 1; }
tail -1 gpurun_out/f_pytest.log
for r in 1 2 3; do for v in 2 6; do
  timeout -k 10 120 python -u tools/small_b_trace.py --graph --opt conv_ring9=$v > gpurun_out/ring9_$v.log 2>&1 || { tail -5 gpurun_out/ring9_$v.log; exit 1; }
  echo "conv_ring9=$v $(tail -1 gpurun_out/ring9_$v.log)"
done; done
timeout -k 10 240 python -u tools/ref_latency.py > gpurun_out/ref_latency.txt 2>&1 || { tail -5 gpurun_out/ref_latency.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/ref_latency.txt
