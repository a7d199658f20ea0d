#!/bin/bash
# Same-box A/B of the working tree's library against libfac_cvit_base.so
# (tools/build_base_lib.sh REF): per-layer times (tools/conv_sweep.py), then
# the CViT bench line, alternating.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
for v in base new base new; do
  if [ $v = base ]; then export FAC_CVIT_LIB=$R/fac_fake_amd/libfac_cvit_base.so; else unset FAC_CVIT_LIB; fi
  timeout -k 10 200 python -u tools/conv_sweep.py --layers ${LAYERS:-3,4,5,6,7,8,13,14,15,16} --tag $v > gpurun_out/sweep_$v.log 2>&1 || { tail -5 gpurun_out/sweep_$v.log; exit 1; }
  tail -1 gpurun_out/sweep_$v.log
done
REPS=${REPS:-2} bash tools/lib_ab.sh
