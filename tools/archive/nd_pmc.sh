#!/bin/bash
# Timings and PMC passes over the convnd_igemm layers of tools/nd_layers.py
# (every layer in one process per pass; dispatches map to layers in order).
# GPU box only: bash tools/nd_pmc.sh [tag]
R=${GRAFT_REPO_ROOT:-$(pwd)}
T=${1:-a}
OUT=$R/gpurun_out/ndpmc_$T
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -k 10 240 python3 -u $R/tools/nd_layers.py --reps 10 > $OUT/times.txt 2>&1 || { tail -5 $OUT/times.txt; exit 1; }
cat $OUT/times.txt
for t in 1 2 3; do
  FAC_ND_TILE=$t timeout -k 10 240 python3 -u $R/tools/nd_layers.py --reps 10 --no-torch > $OUT/times_tile$t.txt 2>&1 || { tail -5 $OUT/times_tile$t.txt; exit 1; }
done
[ -n "$NOPMC" ] && exit 0
PASSES=(
 "FETCH_SIZE TCC_HIT_sum"
 "WRITE_SIZE TCC_MISS_sum"
 "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"
 "TA_TA_BUSY TA_ADDR_STALLED_BY_TC_CYCLES TD_TD_BUSY TCP_PENDING_STALL_CYCLES TCP_TCR_TCP_STALL_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_MFMA"
)
i=0
for p in "${PASSES[@]}"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $p --output-format csv -d $OUT/p$i -o run -- python3 $R/tools/nd_layers.py --reps 3 --no-torch > $OUT/p$i.log 2>&1 || { tail -5 $OUT/p$i.log; exit 1; }
  echo "pass $i ok"
done
