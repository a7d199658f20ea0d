#!/bin/bash
# convnd_pt with LDS-resident biases: GPU op tests, config 5 and 4 bench lines
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py -x -q --timeout 200 --timeout-method thread > gpurun_out/ptb_tests.log 2>&1 || { tail -30 gpurun_out/ptb_tests.log; exit 1; }
tail -1 gpurun_out/ptb_tests.log
REPS=2 bash tools/rvk_ab.sh "FAC_RVK_DUAL=1" || exit 1
REPS=1 WORKLOAD=s3d bash tools/rvk_ab.sh "FAC_ND_PT=1"
