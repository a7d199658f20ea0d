#!/bin/bash
# convnd_pt: GPU op tests, per-layer timings by FAC_ND_PT arm, then config 4/5 bench arms
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pt_tests.log 2>&1 || { tail -30 gpurun_out/pt_tests.log; exit 1; }
tail -1 gpurun_out/pt_tests.log
for a in 0 1 128 256; do FAC_ND_PT=$a timeout -k 10 240 python3 -u tools/nd_layers.py --reps 10 --no-torch > gpurun_out/nd_pt$a.txt 2>&1 || { tail -5 gpurun_out/nd_pt$a.txt; exit 1; }; done
REPS=2 bash tools/rvk_ab.sh "FAC_ND_PT=1" "FAC_ND_PT=0" "FAC_ND_PT=128" || exit 1
REPS=1 WORKLOAD=s3d bash tools/rvk_ab.sh "FAC_ND_PT=1" "FAC_ND_PT=0"
