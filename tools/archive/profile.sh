#!/bin/bash
# GPU-box profiling: rocprofv3 kernel trace + stats, then separate PMC passes
# for HBM traffic (FETCH_SIZE, WRITE_SIZE; MI355X_MICROARCH.md HBM section).
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/prof${PROF_TAG}
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
ARGS="--steps 10 --warmup 3 --no-cpu-baseline ${BENCH_ARGS}"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 $R/bench.py $ARGS > $OUT/trace_bench.log 2>&1 || exit $?
echo trace ok
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- python3 $R/bench.py $ARGS > $OUT/fetch_bench.log 2>&1 || exit $?
echo fetch ok
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- python3 $R/bench.py $ARGS > $OUT/write_bench.log 2>&1 || exit $?
echo write ok
