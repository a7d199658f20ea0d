#!/bin/bash
# SQ counter passes over the bench's stem224 launches (rocprofv3 kernel filter).
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/spmc
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
PASSES=(
 "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES"
 "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU"
)
i=0
for p in "${PASSES[@]}"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $p --kernel-include-regex "stem224" --output-format csv -d $OUT/p$i -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-pipeline --no-graph > $OUT/p$i.log 2>&1 || exit $?
  echo "pass $i ok"
done
