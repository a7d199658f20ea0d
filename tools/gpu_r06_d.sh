#!/bin/bash
# Round 6: the 64x128 encoder GEMM default -- GEMM/tail parity tests, the
# headline against the old tile, configs 5 / RepBn8 against the round-5 lib.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "gemm or few_crop or tail or golden or pipelined or resvitkan or repbn8" > gpurun_out/d_pytest.log 2>&1 || { grep -E "FAILED|Error|error" gpurun_out/d_pytest.log | head -20; tail -5 gpurun_out/d_pytest.log; exit 1; }
tail -1 gpurun_out/d_pytest.log
ARMS="gemm_qkv=-1;gemm_qkv=2 gemm_out=2 gemm_ff1=2 gemm_ff2=2 gemm_head=2" REPS=2 DTYPES="fp16 bf16" STEPS=40 bash tools/ab_bench.sh || exit 1
PREV=ab/libfac_cvit_r05.so ONLY=resvitkan REPS=2 bash tools/lib_ab.sh || exit 1
PREV=ab/libfac_cvit_r05.so ONLY=repbn8 REPS=2 bash tools/lib_ab.sh || exit 1
