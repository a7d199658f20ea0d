#!/bin/bash
# Round 6: barrier ablation (tools/abl_lib.py nobar: WRONG results, timing
# only) of the conv layers at few crops, against the in-tree lib.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
for B in 29 8; do
for rep in 1 2; do
for arm in base nobar; do
  if [ $arm = base ]; then unset FAC_CVIT_LIB; else export FAC_CVIT_LIB=ab/libfac_abl_$arm.so; fi
  timeout -k 10 200 python -u tools/conv_sweep.py --dtype fp16 --B $B --layers 3,4,5,6,7,8,9,10,11,12,13,14,15,16 --tag "$arm B$B" > gpurun_out/ablS_${arm}_$B.txt 2>&1 || { tail -5 gpurun_out/ablS_${arm}_$B.txt; exit 1; }
  tail -1 gpurun_out/ablS_${arm}_$B.txt
done; done; done
