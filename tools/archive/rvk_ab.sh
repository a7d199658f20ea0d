#!/bin/bash
# ResVitKan bench arms (env settings given as arguments, e.g. "FAC_RVK_SIDE=0"
# "FAC_ND_TILE=2"), interleaved over REPS rounds in separate processes on one box.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
W=${WORKLOAD:-resvitkan}
for rep in $(seq 1 ${REPS:-2}); do for arm in "$@"; do
  env $arm timeout -k 10 200 python -u bench.py --only $W --steps 10 --warmup 3 > gpurun_out/rvkab.log 2>&1 || { tail -5 gpurun_out/rvkab.log; exit 1; }
  python -c "import json; l=json.loads(open('gpurun_out/rvkab.log').read().strip().splitlines()[-1]); print('$arm', l['value'], l['ms_per_step'], l['conv_pool_layer_roofline']['fraction_of_step'])"
done; done
