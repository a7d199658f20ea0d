#!/bin/bash
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -m gpu -x -q --timeout 120 --timeout-method thread -k "tk2 or conv_nd_vs_torch" > gpurun_out/tk4_pytest.log 2>&1 || { tail -30 gpurun_out/tk4_pytest.log; exit 1; }
tail -1 gpurun_out/tk4_pytest.log
PREV=ab/libfac_cvit_head.so ONLY=s3d REPS=${REPS:-2} TESTK=s3d bash tools/lib_ab.sh || exit 1
