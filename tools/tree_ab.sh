#!/bin/bash
# Same-box A/B of a previous round's whole tree (Python + its library, e.g.
# ab/r04tree: bench.py, fac_fake_amd/ with libfac_cvit.so) against HEAD on
# one bench sub-measurement, alternating, REPS rounds.
#   PREVTREE=ab/r04tree ONLY=resvitkan REPS=3 bash tools/tree_ab.sh
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
unset FAC_CVIT_LIB
for rep in $(seq 1 ${REPS:-3}); do
  for arm in prev cur; do
    if [ $arm = prev ]; then D=$R/$PREVTREE; else D=$R; fi
    (cd $D && timeout -k 10 300 python -u bench.py --only $ONLY --steps ${STEPS:-10} --warmup 3) > gpurun_out/tab_${ONLY}_${arm}_$rep.log 2>&1 || { tail -5 gpurun_out/tab_${ONLY}_${arm}_$rep.log; exit 1; }
    python - gpurun_out/tab_${ONLY}_${arm}_$rep.log $arm <<'PY'
import json,sys
l=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r=l.get('conv_pool_layer_roofline',{})
print('%-5s %10.1f %s  ms/step %.3f  frac %s' % (sys.argv[2], l['value'], l['unit'], l['ms_per_step'], r.get('fraction_of_step')))
PY
  done
done
