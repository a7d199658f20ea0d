#!/bin/bash
# Round-5 profiles: the headline (bf16) trace + PMC passes, then the fp16
# line with the 14^2 convs as Winograd (option wino=1): trace + SQ passes.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
PROF_TAG=a bash tools/profile_r05.sh || exit 1
OUT=$R/gpurun_out/prof_r05w
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
ARGS="--steps 10 --warmup 3 --dtype fp16 --no-cpu-baseline --no-fp16-line --no-video --no-s3d --no-resvitkan --no-repbn8 --opt wino=1"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 $R/bench.py $ARGS > $OUT/trace_bench.log 2>&1 || exit $?
echo wino trace ok
timeout -s KILL 180 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE --output-format csv -d $OUT/pmc1 -o run -- python3 $R/bench.py $ARGS > $OUT/pmc1_bench.log 2>&1 || exit $?
echo wino pmc1 ok
timeout -s KILL 180 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE --output-format csv -d $OUT/pmc2 -o run -- python3 $R/bench.py $ARGS > $OUT/pmc2_bench.log 2>&1 || exit $?
echo wino pmc2 ok
