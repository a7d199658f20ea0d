#!/bin/bash
# Same-box A/B of a sub-measurement (bench.py --only $1) between environment
# settings (remaining args, "VAR=value" or "-"), alternating, 3 rounds.
mkdir -p gpurun_out
w=$1; shift
for rep in 1 2 3; do
  for arm in "$@"; do
    if [ "$arm" = "-" ]; then envs=""; else envs="$arm"; fi
    env $envs timeout -k 10 200 python bench.py --only $w --steps 20 --warmup 5 > gpurun_out/env_only.log 2>&1 || { echo "[$arm] failed"; tail -3 gpurun_out/env_only.log; exit 1; }
    python -c "import json; d=json.loads(open('gpurun_out/env_only.log').read().strip().splitlines()[-1]); print('[$arm]', d['value'], d['ms_per_step'])"
  done
done
