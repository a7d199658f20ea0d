set -e
for i in 0 1 2 3; do timeout -k 10 60 tools/ubench/bin/nd_ubench $i; done > gpurun_out/nd_ubench_il.txt 2>&1
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py -x -q --timeout 200 --timeout-method thread > gpurun_out/il_tests.log 2>&1 || { tail -30 gpurun_out/il_tests.log; exit 1; }
tail -1 gpurun_out/il_tests.log
for il in 1 0; do FAC_ND_IL=$il timeout -k 10 240 python3 -u tools/nd_layers.py --reps 10 --no-torch > gpurun_out/nd_il$il.txt 2>&1; done
REPS=2 bash tools/rvk_ab.sh "FAC_ND_IL=1" "FAC_ND_IL=0" "FAC_ND_IL=1 FAC_ND_TILE=2"
