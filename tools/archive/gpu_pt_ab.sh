#!/bin/bash
# convnd_pt changes: the GPU op / model tests, then configs 5 and 4 against
# libfac_cvit_base.so, alternating (REPS times).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_pt.log 2>&1 || { grep -E "FAILED|Error|assert" gpurun_out/pytest_pt.log | head -20; tail -3 gpurun_out/pytest_pt.log; exit 1; }
tail -1 gpurun_out/pytest_pt.log
for rep in $(seq ${REPS:-2}); do for v in base new; do
  if [ $v = base ]; then export FAC_CVIT_LIB=$R/fac_fake_amd/libfac_cvit_base.so; else unset FAC_CVIT_LIB; fi
  for w in ${WORKLOADS:-resvitkan s3d}; do
    timeout -k 10 300 python -u bench.py --only $w --steps 10 --warmup 3 > gpurun_out/ab_${w}_$v.log 2>&1 || { tail -5 gpurun_out/ab_${w}_$v.log; exit 1; }
    python -c "import json; l=json.loads(open('gpurun_out/ab_${w}_$v.log').read().strip().splitlines()[-1]); r=l.get('conv_pool_layer_roofline',{}); print('$w $v', l['value'], l['ms_per_step'], r.get('fraction_of_step'))"
  done
done; done
