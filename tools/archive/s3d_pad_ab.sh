#!/bin/bash
# Same-box A/B of S3D (config 4) by FAC_S3D_PAD64 level (0: no channel padding
# of the merged Inception heads, 1: branch1.0 when >= 64, 2: branch2.0 too).
mkdir -p gpurun_out
for rep in 1 2; do
  for arm in FAC_S3D_PAD64=1 FAC_S3D_PAD64=0 FAC_S3D_PAD64=2; do
    env $arm timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --only s3d > gpurun_out/s3d_pad.log 2>&1 || { echo "arm $arm failed"; tail -5 gpurun_out/s3d_pad.log; exit 1; }
    python - "$arm" <<'PY'
import json, sys
d = json.loads(open("gpurun_out/s3d_pad.log").read().strip().splitlines()[-1])
c = d.get("config4", d)
print(f"[{sys.argv[1]}] {c['value']:9.1f} clips/s  {c['ms_per_step']:.3f} ms  layer-roofline frac {c.get('conv_pool_layer_roofline', {}).get('fraction_of_step')}", flush=True)
PY
  done
done
