#!/bin/bash
# round 5: conv_sc1 A/B, few-row GEMM ring variants at B = 29, kernel trace of the B = 29 forward
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
ARMS="conv_sc1=0;conv_sc1=1;conv_sc1=3;conv_sc1=15" TESTK="write_through or each_conv_kernel or gemm_tile_variants or gemm_variants" bash tools/ab_bench.sh || exit 1
for v in 5 7 8 5 7 8; do
  timeout -k 10 120 python -u tools/small_b_trace.py --graph --opt gemm_small=$v > gpurun_out/smallb_$v.log 2>&1 || { tail -5 gpurun_out/smallb_$v.log; exit 1; }
  echo "gemm_small=$v $(tail -1 gpurun_out/smallb_$v.log)"
done
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_small -o small -- python tools/small_b_trace.py > gpurun_out/prof_small.log 2>&1 || { tail -5 gpurun_out/prof_small.log; exit 1; }
tail -1 gpurun_out/prof_small.log
timeout -k 10 120 python -u tools/conv14_nd_ab.py > gpurun_out/nd14.log 2>&1 && timeout -k 10 120 python -u tools/conv14_nd_ab.py --h 28 --cin 256 --cout 256 >> gpurun_out/nd14.log 2>&1 && timeout -k 10 120 python -u tools/conv14_nd_ab.py --h 56 --cin 128 --cout 128 >> gpurun_out/nd14.log 2>&1 || { tail -5 gpurun_out/nd14.log; exit 1; }
grep -v amdgpu gpurun_out/nd14.log
