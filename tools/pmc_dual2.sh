# PMC passes over tools/dual2_ab.py (pw_dual2 vs convnd_pt DUAL at 3072 crops):
# HBM fetch / write bytes and the SQ wait / issue counters per kernel.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/pmc_dual2
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
i=0
for p in "FETCH_SIZE" "WRITE_SIZE" "SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $p --output-format csv -d $OUT/p$i -o run -- python3 $R/tools/dual2_ab.py --rounds 1 --iters 3 > $OUT/p$i.log 2>&1 || { tail -5 $OUT/p$i.log; exit 1; }
  echo "pass $i ok"
done
