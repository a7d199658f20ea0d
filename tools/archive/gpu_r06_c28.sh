#!/bin/bash
# Round 6: the 28x28 layers on 14x14 boxes / 2 x 2 LDS ring (option
# conv28_grid): bit-identity tests, per-layer times of conv10-13 at B = 256
# (both dtypes, two alternations), then the headline line per arm.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "conv28_grid or conv14_grid" > gpurun_out/c28_pytest.log 2>&1 || { grep -E "FAILED|Error|error" gpurun_out/c28_pytest.log | head -20; tail -5 gpurun_out/c28_pytest.log; exit 1; }
tail -1 gpurun_out/c28_pytest.log
for rep in 1 2; do
for g in 0 1 2 3; do
for dt in fp16 bf16; do
  timeout -k 10 200 python -u tools/conv_sweep.py --dtype $dt --layers 9,10,11,12 --opt conv28_grid=$g --tag "$dt g$g" > gpurun_out/c28_${dt}_$g.txt 2>&1 || { tail -5 gpurun_out/c28_${dt}_$g.txt; exit 1; }
  tail -1 gpurun_out/c28_${dt}_$g.txt
done; done; done
ARMS="conv28_grid=0;conv28_grid=1;conv28_grid=3" REPS=2 bash tools/ab_bench.sh
