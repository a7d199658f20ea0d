#!/bin/bash
# fused downsample (fac_conv_nd_dual): GPU op + ResVitKan tests, then config-5 arms
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py -x -q --timeout 200 --timeout-method thread > gpurun_out/dual_tests.log 2>&1 || { tail -30 gpurun_out/dual_tests.log; exit 1; }
tail -1 gpurun_out/dual_tests.log
REPS=2 bash tools/rvk_ab.sh "FAC_RVK_DUAL=1" "FAC_RVK_DUAL=0" || exit 1
timeout -k 10 200 python3 -u tools/rvk_layers.py --model rvk --B 512 > gpurun_out/rvk_layers_dual.txt 2>&1
