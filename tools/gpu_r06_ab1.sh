#!/bin/bash
# Round 6: same-box A/Bs -- configs 4/5 of the round-4 tree against HEAD
# (VERDICT r05 item 5), the round-5 library against HEAD on the headline
# (item 6), and the GEMM reference points.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/gemm_ceiling.py > gpurun_out/gemm_ceiling2.txt 2>&1 || { tail -5 gpurun_out/gemm_ceiling2.txt; exit 1; }
grep -E "^(square|conv15_tap|conv11_tap)" gpurun_out/gemm_ceiling2.txt
PREVTREE=ab/r04tree ONLY=resvitkan REPS=3 bash tools/tree_ab.sh || exit 1
PREVTREE=ab/r04tree ONLY=s3d REPS=2 bash tools/tree_ab.sh || exit 1
PREV=ab/libfac_cvit_r05.so DTYPES="bf16 fp16" REPS=2 bash tools/lib_ab_cvit.sh || exit 1
