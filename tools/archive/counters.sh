#!/bin/bash
# PMC passes (each its own rocprofv3 run) over a short bench; args: counter groups separated by ';'
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/pmc
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
rocprofv3 -L > $OUT/counters_list.txt 2>&1 || true
i=0
IFS=';' read -ra PASSES <<< "$1"
for g in "${PASSES[@]}"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $g --output-format csv -d $OUT/p$i -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-graph ${BENCH_ARGS} > $OUT/p$i.log 2>&1 || exit $?
  echo "pass $i ok: $g"
done
