#!/bin/bash
# GPU-box: rocprofv3 trace + FETCH/WRITE passes for the CViT headline (config 2)
# and trace-only passes for the config-4 / config-5 sub-measurements.
R=${GRAFT_REPO_ROOT:-$(pwd)}
BENCH_ARGS="--no-video --no-resvitkan --no-s3d --no-repbn8" PROF_TAG=_cvit bash $R/tools/profile.sh || exit $?
export TMPDIR=/tmp
cd /tmp
for w in resvitkan s3d repbn8; do
  mkdir -p $R/gpurun_out/prof_$w
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_$w/trace -o run -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --only $w > $R/gpurun_out/prof_$w/trace_bench.log 2>&1 || exit $?
  echo $w ok
done
