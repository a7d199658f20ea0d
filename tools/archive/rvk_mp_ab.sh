#!/bin/bash
# Same-box A/B of ResVitKan (config 5) with conv1 + maxpool fused
# (conv_s2d4_mp, default) vs conv_s2d4 then fac_pool_nd (FAC_RVK_MP=0).
mkdir -p gpurun_out
for rep in 1 2; do
  for arm in FAC_RVK_MP=1 FAC_RVK_MP=0; do
    env $arm timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --only resvitkan > gpurun_out/rvk_mp.log 2>&1 || { echo "arm $arm failed"; tail -5 gpurun_out/rvk_mp.log; exit 1; }
    python - "$arm" <<'PY'
import json, sys
d = json.loads(open("gpurun_out/rvk_mp.log").read().strip().splitlines()[-1])
c = d.get("config5", d)
print(f"[{sys.argv[1]}] {c['value']:9.1f} crops/s  {c['ms_per_step']:.3f} ms  layer-roofline frac {c.get('conv_pool_layer_roofline', {}).get('fraction_of_step')}", flush=True)
PY
  done
done
