#!/bin/bash
# S3D max-pool kernels, same process family, same box: config 4 with
# fac_set_option pool_impl = 0 (pool_nd / maxpool3_s1), 1 (maxpool_fixed),
# 2 (maxpool3_lds), 3 (both), alternating.  (Round 4: the two kernels and
# the pool_impl option were removed after this A/B; kept as
# the record of how it was measured.)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
for rep in 1 2; do for a in ${ARMS:-0 1 2 3}; do
  timeout -k 10 300 python -u bench.py --only s3d --steps 10 --warmup 3 --opt pool_impl=$a > gpurun_out/pool_$a.log 2>&1 || { tail -5 gpurun_out/pool_$a.log; exit 1; }
  python -c "import json; l=json.loads(open('gpurun_out/pool_$a.log').read().strip().splitlines()[-1]); print('pool_impl=$a', l['value'], l['ms_per_step'])"
done; done
