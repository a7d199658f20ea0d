#!/bin/bash
# few-crop 14^2 convs on 32-channel blocks (option conv_small14 1 / 0): bit-identity tests, then graph forwards at B = 1 / 8 / 16 / 29
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "small14 or ring9 or few_crop or small_batch_graph" > gpurun_out/s14_pytest.log 2>&1 || { tail -30 gpurun_out/s14_pytest.log; exit 1; }
tail -1 gpurun_out/s14_pytest.log
for rep in 1 2; do
  for v in 0 1; do
    for b in 1 8 16 29; do
      echo -n "conv_small14=$v "; timeout -k 10 120 python -u tools/small_b_trace.py --graph --batch $b --reps 300 --warmup 200 --opt conv_small14=$v 2>&1 | grep -v amdgpu.ids | tail -1 || exit 1
    done
  done
done
timeout -k 10 240 python -u tools/ref_latency.py 2>&1 | grep -v amdgpu.ids | grep "predict_video\|B=29 graph (device"
