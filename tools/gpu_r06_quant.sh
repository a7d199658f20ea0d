#!/bin/bash
# Round 6: per-layer time vs batch (wave quantisation of each conv grid).
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
for B in 256 128 192 219 240 272 292 320 256; do
  timeout -k 10 120 python -u tools/conv_sweep.py --B $B > gpurun_out/quant_$B.log 2>&1 || { tail -5 gpurun_out/quant_$B.log; exit 1; }
  tail -1 gpurun_out/quant_$B.log | cut -c1-400
done
