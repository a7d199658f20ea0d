#!/bin/bash
# Round 6: config-4 / config-5 kernel-time breakdown at the bench batches
# (kernel trace + stats of `bench.py --only s3d|resvitkan`).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
export TMPDIR=/tmp
cd /tmp
for w in s3d resvitkan; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof6_$w -o run -- python3 $R/bench.py --steps 5 --warmup 2 --only $w > $R/gpurun_out/prof6_$w.log 2>&1 || { tail -5 $R/gpurun_out/prof6_$w.log; exit 1; }
  echo $w ok
done
