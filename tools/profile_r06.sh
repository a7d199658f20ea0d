#!/bin/bash
# GPU-box profiling of the config-2 CViT forward (bench.py, bf16 unless
# DTYPE=fp16): rocprofv3 kernel trace + stats, then one rocprofv3 run per PMC
# pass (MI355X_MICROARCH.md: counters are not split over passes; FETCH_SIZE and
# WRITE_SIZE do not fit one TCC pass).  Summarise with
#   python tools/rocprof_summary.py gpurun_out/prof_r06 profiles/r06_bf16
R=${GRAFT_REPO_ROOT:-$(pwd)}
DT=${DTYPE:-bf16}
OUT=$R/gpurun_out/prof_r06${PROF_TAG}
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
ARGS="--steps 10 --warmup 3 --dtype $DT --no-cpu-baseline --no-fp16-line --no-video --no-s3d --no-resvitkan --no-repbn8 ${BENCH_ARGS}"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 $R/bench.py $ARGS > $OUT/trace_bench.log 2>&1 || exit $?
echo trace ok
run_pmc() {  # name, counters
  timeout -s KILL 180 rocprofv3 --pmc $2 --output-format csv -d $OUT/$1 -o run -- python3 $R/bench.py $ARGS > $OUT/$1_bench.log 2>&1 || exit $?
  echo "$1 ok"
}
run_pmc fetch "FETCH_SIZE"
run_pmc write "WRITE_SIZE"
run_pmc pmc1 "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"
run_pmc pmc2 "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE"
