#!/bin/bash
# Same-box FETCH_SIZE / WRITE_SIZE of the CViT forward with the round-4 tree
# (ab/r04tree: its bench.py + library) and HEAD, alternating (VERDICT r05
# item 4: conv6's HBM bytes rose 746 -> 846 MB between r04c and r05z).
# Summarise with tools/rocprof_summary.py per arm.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
unset FAC_CVIT_LIB
ARGS="--steps 10 --warmup 3 --dtype bf16 --no-cpu-baseline --no-fp16-line --no-video --no-s3d --no-resvitkan --no-repbn8"
for rep in 1 2; do
  for arm in prev cur; do
    if [ $arm = prev ]; then D=$R/ab/r04tree; else D=$R; fi
    OUT=$R/gpurun_out/c6f_${arm}_$rep
    mkdir -p $OUT
    cd /tmp
    timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- python3 $D/bench.py $ARGS > $OUT/fetch_bench.log 2>&1 || exit $?
    timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- python3 $D/bench.py $ARGS > $OUT/write_bench.log 2>&1 || exit $?
    echo "$arm $rep ok"
  done
done
