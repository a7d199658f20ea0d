#!/bin/bash
# Round 6: kernel trace of the pipelined headline with the pre-deferral lib.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
export TMPDIR=/tmp
export FAC_CVIT_LIB=$R/ab/libfac_cvit_predefer.so
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/prof6_pipe_pre -o run -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-fp16-line --no-video --no-s3d --no-resvitkan --no-repbn8 > $R/gpurun_out/prof6_pipe_pre.log 2>&1 || { tail -5 $R/gpurun_out/prof6_pipe_pre.log; exit 1; }
tail -1 $R/gpurun_out/prof6_pipe_pre.log | cut -c1-200
