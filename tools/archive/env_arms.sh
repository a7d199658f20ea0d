#!/bin/bash
# Same-box bench arms that differ by environment: each argument is "VAR=value"
# (or "-" for none); prints crops/s and per-stage groups, twice, alternating.
mkdir -p gpurun_out
for rep in 1 2; do
  for arm in "$@"; do
    if [ "$arm" = "-" ]; then envs=""; else envs="$arm"; fi
    env $envs timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-video --no-s3d --no-resvitkan --no-repbn8 > gpurun_out/arm.log 2>&1 || { echo "arm [$arm] failed"; tail -5 gpurun_out/arm.log; exit 1; }
    python - "$arm" <<'PY'
import json, sys
d = json.loads(open("gpurun_out/arm.log").read().strip().splitlines()[-1])
st = d["stage_ms"]
g = lambda a, b: sum(st[f"conv{i}"] for i in range(a, b + 1))
print(f"[{sys.argv[1]:16s}] {d['value']:9.1f} crops/s  {d['ms_per_step']:.3f} ms  conv4-6 {g(4, 6):.3f} "
      f"56^2 {g(7, 9):.3f} 28^2 {g(10, 13):.3f} 14^2 {g(14, 17):.3f}", flush=True)
PY
  done
done
