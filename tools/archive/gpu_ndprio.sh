#!/bin/bash
# A/B: convnd_pt static priority (option nd_prio) on configs 5 and 4
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "resvitkan_matches or conv_nd_pt or conv_dual or s3d_matches" > gpurun_out/ndp_pytest.log 2>&1 || { tail -30 gpurun_out/ndp_pytest.log; exit 1; }
tail -1 gpurun_out/ndp_pytest.log
for rep in 1 2; do
  for only in resvitkan s3d; do
    for v in 0 1 2; do
      timeout -k 10 300 python -u bench.py --only $only --steps 10 --warmup 3 --opt nd_prio=$v > gpurun_out/ndp_${only}_${v}_$rep.log 2>&1 || { tail -5 gpurun_out/ndp_${only}_${v}_$rep.log; exit 1; }
      python - gpurun_out/ndp_${only}_${v}_$rep.log $only $v <<'PY'
import json,sys
l=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r=l.get('conv_pool_layer_roofline',{})
print('%-9s nd_prio=%s %10.1f %s  ms/step %.3f  frac %s' % (sys.argv[2], sys.argv[3], l['value'], l['unit'], l['ms_per_step'], r.get('fraction_of_step')))
PY
    done
  done
done
