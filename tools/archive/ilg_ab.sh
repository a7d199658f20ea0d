#!/bin/bash
# interleaved glds issue on convnd_igemm's general gather: op + S3D tests, then config-4 arms
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py -x -q --timeout 200 --timeout-method thread > gpurun_out/ilg_tests.log 2>&1 || { tail -30 gpurun_out/ilg_tests.log; exit 1; }
tail -1 gpurun_out/ilg_tests.log
REPS=2 WORKLOAD=s3d bash tools/rvk_ab.sh "FAC_ND_IL_G=1" "FAC_ND_IL_G=0"
