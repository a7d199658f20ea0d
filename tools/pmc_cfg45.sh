#!/bin/bash
# PMC passes over the eager config-4 (S3D, 256 uint8 clips: base.0 as one
# launch) and config-5 (ResVitKan, 512 crops) forwards of tools/rvk_layers.py:
# MFMA busy, LDS and wave-state counters in one pass, FETCH_SIZE and
# WRITE_SIZE in passes of their own (MI355X_MICROARCH.md: one block budget per
# run).  GPU box only; summarise with
#   python tools/pmc_cfg45_summary.py gpurun_out/pmc_cfg45<TAG> profiles/<prefix>
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/pmc_cfg45${PROF_TAG}
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
PASSES=(
 "SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"
 "FETCH_SIZE"
 "WRITE_SIZE"
)
for m in s3d rvk; do
  B=256; X="--u8"; [ $m = rvk ] && { B=512; X=""; }
  i=0
  for p in "${PASSES[@]}"; do
    i=$((i+1))
    timeout -s KILL 150 rocprofv3 --pmc $p --output-format csv -d $OUT/${m}_p$i -o run -- python3 $R/tools/rvk_layers.py --model $m --B $B --reps 1 $X > $OUT/${m}_p$i.log 2>&1 || { tail -5 $OUT/${m}_p$i.log; exit 1; }
    echo "$m pass $i ok"
  done
done
