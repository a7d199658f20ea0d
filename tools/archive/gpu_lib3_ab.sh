#!/bin/bash
# Three-library A/B on one box: libfac_cvit_base.so, libfac_cvit.so (new),
# libfac_cvit_alt.so (alt); bench sub-measurements WORKLOADS, alternating.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
[ -n "$TESTS" ] && { timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "$TESTS" > gpurun_out/pytest_lib3.log 2>&1 || { grep -E "FAILED|Error|assert" gpurun_out/pytest_lib3.log | head -20; tail -3 gpurun_out/pytest_lib3.log; exit 1; }; tail -1 gpurun_out/pytest_lib3.log; }
for rep in $(seq ${REPS:-2}); do for v in base new alt; do
  case $v in base) export FAC_CVIT_LIB=$R/fac_fake_amd/libfac_cvit_base.so;; alt) export FAC_CVIT_LIB=$R/fac_fake_amd/libfac_cvit_alt.so;; *) unset FAC_CVIT_LIB;; esac
  for w in ${WORKLOADS:-resvitkan}; do
    timeout -k 10 300 python -u bench.py --only $w --steps 10 --warmup 3 > gpurun_out/ab3_${w}_$v.log 2>&1 || { tail -5 gpurun_out/ab3_${w}_$v.log; exit 1; }
    python -c "import json; l=json.loads(open('gpurun_out/ab3_${w}_$v.log').read().strip().splitlines()[-1]); r=l.get('conv_pool_layer_roofline',{}); print('$w $v', l['value'], l['ms_per_step'], r.get('fraction_of_step'))"
  done
done; done
