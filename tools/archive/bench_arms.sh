#!/bin/bash
# Same-box bench arms: each argument is one set of bench.py flags; prints
# crops/s, ms/step and the per-stage groups for every arm, twice (alternating).
mkdir -p gpurun_out
for rep in 1 2; do
  for arm in "$@"; do
    timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-video --no-s3d --no-resvitkan --no-repbn8 $arm > gpurun_out/arm.log 2>&1 || { echo "arm [$arm] failed"; tail -5 gpurun_out/arm.log; exit 1; }
    python - "$arm" <<'PY'
import json, sys
d = json.loads(open("gpurun_out/arm.log").read().strip().splitlines()[-1])
st = d["stage_ms"]
groups = {"stem": ["conv1"], "112": ["conv4", "conv5", "conv6"], "56": ["conv7", "conv8", "conv9"],
          "28": ["conv10", "conv11", "conv12", "conv13"], "14": ["conv14", "conv15", "conv16", "conv17"],
          "tail": ["patch_embed", "transformer", "head"]}
g = {k: round(sum(st[s] for s in v), 3) for k, v in groups.items()}
print(f"[{sys.argv[1]:28s}] {d['value']:9.1f} crops/s  {d['ms_per_step']:.3f} ms  stem {d['roofline']['launch_ms']:.3f}  {g}", flush=True)
PY
  done
done
