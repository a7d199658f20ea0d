#!/bin/bash
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -k "fused_attention or few_crop or graph or weights_changed or ring9 or tail" > gpurun_out/g_pytest.log 2>&1 || { tail -30 gpurun_out/g_pytest.log; exit 1; }
tail -1 gpurun_out/g_pytest.log
for r in 1 2 3; do for v in 1 0; do
  timeout -k 10 120 python -u tools/small_b_trace.py --graph --opt attn_fuse=$v > gpurun_out/af_$v.log 2>&1 || { tail -5 gpurun_out/af_$v.log; exit 1; }
  echo "attn_fuse=$v $(tail -1 gpurun_out/af_$v.log)"
done; done
timeout -k 10 240 python -u tools/ref_latency.py > gpurun_out/ref_latency.txt 2>&1 || { tail -5 gpurun_out/ref_latency.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/ref_latency.txt
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 180 rocprofv3 --kernel-trace -d gpurun_out/prof_small_g -o small -- python tools/small_b_trace.py --graph --reps 50 > gpurun_out/prof_small_g.log 2>&1 || { tail -5 gpurun_out/prof_small_g.log; exit 1; }
