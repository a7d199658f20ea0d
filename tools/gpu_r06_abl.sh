#!/bin/bash
# Round 6: ablation arms of conv3x3_bn_relu (tools/abl_lib.py; WRONG results,
# timing only) on the ring-kernel layers at B = 256, against the in-tree lib.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
for rep in 1 2; do
for arm in base w0 now nomfma nobar noA; do
  if [ $arm = base ]; then unset FAC_CVIT_LIB; else export FAC_CVIT_LIB=ab/libfac_abl_$arm.so; fi
  timeout -k 10 200 python -u tools/conv_sweep.py --dtype bf16 --layers 3,4,5,6,7,8,13,14,15,16 --tag "$arm" > gpurun_out/abl_$arm.txt 2>&1 || { tail -5 gpurun_out/abl_$arm.txt; exit 1; }
  tail -1 gpurun_out/abl_$arm.txt
done; done
