#!/bin/bash
# Round 6: the 14x14 / BN-128 wave-grid arms (option conv14_grid): bit-identity
# tests, per-layer times of conv14-17 at B = 256 (both dtypes, two
# alternations), then the headline line per arm.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "conv14_grid or isolated or ring9 or small14 or golden" > gpurun_out/c14_pytest.log 2>&1 || { grep -E "FAILED|Error|error" gpurun_out/c14_pytest.log | head -20; tail -5 gpurun_out/c14_pytest.log; exit 1; }
tail -1 gpurun_out/c14_pytest.log
for rep in 1 2; do
for g in 0 1 2 3 4; do
for dt in fp16 bf16; do
  timeout -k 10 200 python -u tools/conv_sweep.py --dtype $dt --layers 13,14,15,16 --opt conv14_grid=$g --tag "$dt g$g" > gpurun_out/c14_${dt}_$g.txt 2>&1 || { tail -5 gpurun_out/c14_${dt}_$g.txt; exit 1; }
  tail -1 gpurun_out/c14_${dt}_$g.txt
done; done; done
ARMS="conv14_grid=0;conv14_grid=1;conv14_grid=2;conv14_grid=4" REPS=1 bash tools/ab_bench.sh
