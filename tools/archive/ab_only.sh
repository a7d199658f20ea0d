#!/bin/bash
# Same-box A/B of a sub-measurement (bench.py --only $1) between the base
# library (tools/build_base_lib.sh) and the in-tree build, alternating, 3 rounds.
mkdir -p gpurun_out
for rep in 1 2 3; do
  for arm in base tree; do
    if [ $arm = base ]; then export FAC_CVIT_LIB=$(pwd)/fac_fake_amd/libfac_cvit_base.so; else unset FAC_CVIT_LIB; fi
    timeout -k 10 200 python bench.py --only $1 --steps 20 --warmup 5 > gpurun_out/ab_only.log 2>&1 || { echo "$arm failed"; tail -3 gpurun_out/ab_only.log; exit 1; }
    python -c "import json; d=json.loads(open('gpurun_out/ab_only.log').read().strip().splitlines()[-1]); print('$arm', d['value'], d['ms_per_step'])"
  done
done
