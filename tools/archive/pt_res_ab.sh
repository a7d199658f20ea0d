#!/bin/bash
# convnd_pt residual variant: GPU op tests with and without FAC_PW_PT, then config-5 arms
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
for v in 0 1; do
  FAC_PW_PT=$v timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py -x -q --timeout 200 --timeout-method thread > gpurun_out/ptres_tests_$v.log 2>&1 || { tail -30 gpurun_out/ptres_tests_$v.log; exit 1; }
  tail -1 gpurun_out/ptres_tests_$v.log
done
REPS=2 bash tools/rvk_ab.sh "FAC_PW_PT=0" "FAC_PW_PT=1" || exit 1
FAC_PW_PT=1 timeout -k 10 200 python3 -u tools/rvk_layers.py --model rvk --B 512 > gpurun_out/rvk_layers_ptres.txt 2>&1
