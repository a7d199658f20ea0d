#!/bin/bash
# kernel trace of B=29 graph forwards (the reference's one-video call), per-kernel sequence
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
R=$(pwd)
mkdir -p gpurun_out
export TMPDIR=/tmp
(cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace -d $R/gpurun_out/prof_small_h -o small -- python3 $R/tools/small_b_trace.py --graph --reps 100 --warmup 100 > $R/gpurun_out/prof_small_h.log 2>&1) || { tail -5 gpurun_out/prof_small_h.log; exit 1; }
tail -1 gpurun_out/prof_small_h.log
db=$(ls gpurun_out/prof_small_h/*.db gpurun_out/prof_small_h/*/*.db 2>/dev/null | head -1)
python tools/trace_forward.py $db
