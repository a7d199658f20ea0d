#!/bin/bash
# Sustained clock of the fused stem in bf16 vs fp16: GRBM_GUI_ACTIVE / 8 over
# each dispatch's duration (rocprofv3 --pmc, dispatch timestamps from its CSV, one run per
# dtype).  GPU box only; summarise with tools/dtype_clock.py.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/dtype_clock
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
for dt in bf16 fp16; do
  timeout -s KILL 150 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES --output-format csv -d $OUT/$dt -o run -- \
    python3 $R/bench.py --dtype $dt --steps 10 --warmup 3 --no-fp16-line --no-video --no-s3d --no-resvitkan --no-repbn8 --no-cpu-baseline > $OUT/$dt.log 2>&1 || { tail -5 $OUT/$dt.log; exit 1; }
  echo "$dt ok"
done
