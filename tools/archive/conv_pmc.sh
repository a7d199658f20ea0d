#!/bin/bash
# SQ counter passes over single conv layers (tools/conv_sweep.py, hipGraph of
# 20 launches): ./tools/conv_pmc.sh "4 14"; GPU box only.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/cpmc
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
PASSES=(
 "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES"
 "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_MFMA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM"
)
for L in ${1:-4 14}; do for O in ${OPTS:-conv112_persist=4}; do
  i=0
  for p in "${PASSES[@]}"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $p --output-format csv -d $OUT/l${L}${O#*=}_p$i -o run -- python3 $R/tools/conv_sweep.py --layers $L --B 256 --opt $O > $OUT/l${L}${O#*=}_p$i.log 2>&1 || exit $?
  done
  echo "layer $L $O ok"; done
done
