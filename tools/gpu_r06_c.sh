#!/bin/bash
# Round 6: few-row GEMMs with MALL-warm weights (24 MB flush), and the B = 29
# graph forward's per-launch durations (kernel trace).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/gemm_l2.py --dtype fp16 --flush-mb 24 > gpurun_out/gemm_l2_24.txt 2>&1 || { tail -5 gpurun_out/gemm_l2_24.txt; exit 1; }
grep -v "^{" gpurun_out/gemm_l2_24.txt | grep -v amdgpu
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/prof_small -o small -- python3 $R/tools/small_b_trace.py --graph --dtype fp16 --reps 100 --warmup 100 > $R/gpurun_out/prof_small.log 2>&1 || { tail -5 $R/gpurun_out/prof_small.log; exit 1; }
cd $R
DB=$(ls gpurun_out/prof_small/*/small_results.db gpurun_out/prof_small/small_results.db 2>/dev/null | head -1)
python tools/trace_forward.py $DB > gpurun_out/small_fwd_trace.txt 2>&1 || { tail -5 gpurun_out/small_fwd_trace.txt; exit 1; }
tail -70 gpurun_out/small_fwd_trace.txt
