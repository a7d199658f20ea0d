#!/bin/bash
# Round 6: kernel trace of the pipelined headline (timeline of the conv and
# encoder streams), bf16.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/prof6_pipe -o run -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-fp16-line --no-video --no-s3d --no-resvitkan --no-repbn8 > $R/gpurun_out/prof6_pipe.log 2>&1 || { tail -5 $R/gpurun_out/prof6_pipe.log; exit 1; }
tail -1 $R/gpurun_out/prof6_pipe.log | cut -c1-200
