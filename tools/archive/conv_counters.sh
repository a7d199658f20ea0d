#!/bin/bash
# PMC passes over one conv layer (tools/conv_sweep.py), old per-box kernel vs
# persistent kernel: ./tools/conv_counters.sh <layer-index> ; GPU box only.
R=${GRAFT_REPO_ROOT:-$(pwd)}
L=${1:-14}
OUT=$R/gpurun_out/cpmc
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
PASSES=(
 "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES"
 "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_INSTS_MFMA"
 "SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_VALU SQ_INST_LEVEL_LDS SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM SQ_ACTIVE_INST_MISC SQ_INSTS_SALU"
 "TA_TA_BUSY TA_BUFFER_READ_LDS_WAVEFRONTS TA_FLAT_READ_LDS_WAVEFRONTS TA_ADDR_STALLED_BY_TC_CYCLES TA_DATA_STALLED_BY_TC_CYCLES TD_TD_BUSY TCP_PENDING_STALL_CYCLES TCP_TCR_TCP_STALL_CYCLES"
)
i=0
for p in "${PASSES[@]}"; do
  i=$((i+1))
  for v in 0 1; do
    timeout -k 10 300 rocprofv3 --pmc $p --output-format csv -d $OUT/p${i}_v$v -o run -- python3 $R/tools/conv_sweep.py --layers $L --B 256 --opt conv_persist=$v > $OUT/p${i}_v$v.log 2>&1 || exit $?
  done
  echo "pass $i ok"
done
