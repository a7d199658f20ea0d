#!/bin/bash
# Same-box A/B of the in-tree library against a previous build (ab/*.so, via
# FAC_CVIT_LIB) on one bench sub-measurement, alternating, REPS rounds.
#   PREV=ab/libfac_cvit_prev.so ONLY=s3d REPS=3 TESTK=s3d bash tools/lib_ab.sh
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
if [ -n "$TESTK" ]; then
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "$TESTK" > gpurun_out/lab_pytest.log 2>&1 || { tail -30 gpurun_out/lab_pytest.log; exit 1; }
  tail -1 gpurun_out/lab_pytest.log
fi
for rep in $(seq 1 ${REPS:-3}); do
  for arm in prev cur; do
    if [ $arm = prev ]; then export FAC_CVIT_LIB=$PREV; else unset FAC_CVIT_LIB; fi
    timeout -k 10 300 python -u bench.py --only $ONLY --steps ${STEPS:-10} --warmup 3 > gpurun_out/lab_${arm}_$rep.log 2>&1 || { tail -5 gpurun_out/lab_${arm}_$rep.log; exit 1; }
    python - gpurun_out/lab_${arm}_$rep.log $arm <<'PY'
import json,sys
l=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r=l.get('conv_pool_layer_roofline',{})
print('%-5s %10.1f %s  ms/step %.3f  frac %s' % (sys.argv[2], l['value'], l['unit'], l['ms_per_step'], r.get('fraction_of_step')))
PY
  done
done
unset FAC_CVIT_LIB
