#!/bin/bash
# Same-box A/B of ResVitKan (config 5): layer2's conv3 + next conv1 fused
# (bneck_pw2_l2, FAC_RVK_PW2_L2=1) vs two launches (the default).
mkdir -p gpurun_out
for rep in 1 2; do
  for arm in FAC_RVK_PW2_L2=1 FAC_RVK_PW2_L2=0; do
    env $arm timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --only resvitkan > gpurun_out/rvk_pw2l2.log 2>&1 || { echo "arm $arm failed"; tail -5 gpurun_out/rvk_pw2l2.log; exit 1; }
    python - "$arm" <<'PY'
import json, sys
d = json.loads(open("gpurun_out/rvk_pw2l2.log").read().strip().splitlines()[-1])
c = d.get("config5", d)
print(f"[{sys.argv[1]}] {c['value']:9.1f} crops/s  {c['ms_per_step']:.3f} ms  layer-roofline frac {c.get('conv_pool_layer_roofline', {}).get('fraction_of_step')}", flush=True)
PY
  done
done
