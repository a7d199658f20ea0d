#!/bin/bash
# Same-box A/B of the working tree's libfac_cvit.so against fac_fake_amd/libfac_cvit_base.so
# (tools/build_base_lib.sh REF) on the CViT bench, alternating, REPS times.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
ARGS=${ARGS:-"--steps 50 --warmup 10 --no-fp16-line --no-video --no-s3d --no-resvitkan --no-repbn8 --no-cpu-baseline"}
for rep in $(seq ${REPS:-2}); do for v in base new; do
  if [ $v = base ]; then export FAC_CVIT_LIB=$R/fac_fake_amd/libfac_cvit_base.so; else unset FAC_CVIT_LIB; fi
  timeout -k 10 200 python -u bench.py $ARGS > gpurun_out/libab_$v.log 2>&1 || { tail -5 gpurun_out/libab_$v.log; exit 1; }
  python -c "import json,sys; l=json.loads(open('gpurun_out/libab_$v.log').read().strip().splitlines()[-1]); r=l.get('roofline',{}); print('$v', l['value'], l['ms_per_step'], r.get('launch_ms'), r.get('launch_ms_sync_profile'), r.get('frac'))"
done; done
