#!/bin/bash
# A library change to the conv kernels: every GPU test, then same-box A/B of
# the working tree's library against libfac_cvit_base.so (per-layer sweep,
# CViT bench, configs 4/5), alternating.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
NO_BENCH=1 bash tools/gpu_r04.sh || exit 1
LAYERS=${LAYERS:-3,4,5,6,7,8,9,10,11,12,13,14,15,16} bash tools/gpu_libab.sh || exit 1
for v in base new; do
  if [ $v = base ]; then export FAC_CVIT_LIB=$R/fac_fake_amd/libfac_cvit_base.so; else unset FAC_CVIT_LIB; fi
  for w in s3d resvitkan; do
    timeout -k 10 300 python -u bench.py --only $w --steps 10 --warmup 3 > gpurun_out/ab_${w}_$v.log 2>&1 || { tail -5 gpurun_out/ab_${w}_$v.log; exit 1; }
    python -c "import json; l=json.loads(open('gpurun_out/ab_${w}_$v.log').read().strip().splitlines()[-1]); print('$w $v', l['value'], l['ms_per_step'])"
  done
done
