#!/bin/bash
# Same-box A/B of S3D (config 4): SepConv middle channels padded to 64 below
# 14x14 (FAC_S3D_PADT=1) or not.
mkdir -p gpurun_out
for rep in 1 2; do
  for arm in FAC_S3D_PADT=1 FAC_S3D_PADT=0; do
    env $arm timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --only s3d > gpurun_out/s3d_padt.log 2>&1 || { echo "arm $arm failed"; tail -5 gpurun_out/s3d_padt.log; exit 1; }
    python - "$arm" <<'PY'
import json, sys
d = json.loads(open("gpurun_out/s3d_padt.log").read().strip().splitlines()[-1])
c = d.get("config4", d)
print(f"[{sys.argv[1]}] {c['value']:9.1f} clips/s  {c['ms_per_step']:.3f} ms  layer-roofline frac {c.get('conv_pool_layer_roofline', {}).get('fraction_of_step')}", flush=True)
PY
  done
done
