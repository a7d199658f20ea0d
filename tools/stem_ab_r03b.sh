#!/bin/bash
# A/B of stem224_fused (stem_version 0) and stem224_strip (1), same box:
# fused-stem parity tests under each version, the outputs of the two against
# each other, then the CViT-only bench per version (twice).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
FAC_STEM_VERSION=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "fused_stem or conv1_fused or golden or b256 or real_crops or whole" > gpurun_out/r03_stemb_tests.log 2>&1 || { tail -30 gpurun_out/r03_stemb_tests.log; exit 1; }
tail -1 gpurun_out/r03_stemb_tests.log
timeout -k 10 200 python -u - > gpurun_out/r03_stemb_eq.log 2>&1 <<PY || { tail -20 gpurun_out/r03_stemb_eq.log; exit 1; }
import numpy as np, torch, sys
sys.path.insert(0, ".")
from fac_fake_amd import _lib
from fac_fake_amd.cvit import CViT
from fac_fake_amd.weights import make_crops, make_state_dict
lib = _lib.load()
sd = make_state_dict(0)
for dt in ("bf16", "fp16"):
    tdt = torch.bfloat16 if dt == "bf16" else torch.float16
    m = CViT(dtype=dt); m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in sd.items()}); m.to("cuda:0"); m.reserve(8, "cuda:0")
    x = torch.from_numpy(make_crops(6, seed=29)).cuda()
    outs = []
    for v in (0, 1):
        m.set_option("stem_version", v)
        o = torch.empty(6, 112, 112, 32, dtype=tdt, device="cuda:0")
        _lib.check(lib.fac_debug_features_u8(m._ctx, x.data_ptr(), 6, 2, o.data_ptr(), None), m._ctx, "dbg")
        torch.cuda.synchronize()
        outs.append(o.float().cpu())
    d = (outs[0] != outs[1]).float().mean().item()
    rel = ((outs[0] - outs[1]).abs() / outs[0].abs().clamp_min(1e-3)).max().item()
    print(dt, "differing fraction", d, "max rel", rel, flush=True)
    m.set_option("stem_version", 0)
    m._release()
PY
cat gpurun_out/r03_stemb_eq.log | tail -2
for rep in 1 2; do
for v in 0 1; do
  timeout -k 10 200 python -u bench.py --steps 50 --warmup 10 --no-fp16-line --no-video --no-s3d --no-resvitkan --no-repbn8 --no-cpu-baseline --opt stem_version=$v > gpurun_out/r03_stemb_$v.log 2>&1 || { tail -5 gpurun_out/r03_stemb_$v.log; exit 1; }
  python -c "import json,sys; l=json.loads(open('gpurun_out/r03_stemb_$v.log').read().strip().splitlines()[-1]); print('v$v', l['value'], l['ms_per_step'], l['roofline']['launch_ms'], l['roofline']['launch_ms_sync_profile'], l['roofline']['frac'], l['parity']['max_abs_dprob'])"
done
done
