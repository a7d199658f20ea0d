#!/bin/bash
# A/B of the stem kernels, same box: bit-identity of every variant against
# stem224_fused, then bench (CViT only) per stem_version in $VERS (twice).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
VERS=${VERS:-"0 1 2 3 4 5 6 7 8"}
timeout -k 10 200 python -u - > gpurun_out/r03_stemab_eq.log 2>&1 <<PY || { tail -20 gpurun_out/r03_stemab_eq.log; exit 1; }
import numpy as np, torch, sys
sys.path.insert(0, ".")
from fac_fake_amd import _lib
from fac_fake_amd.cvit import CViT
from fac_fake_amd.weights import make_crops, make_state_dict
lib = _lib.load()
sd = make_state_dict(0)
for dt in ("bf16", "fp16"):
    m = CViT(dtype=dt); m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in sd.items()}); m.to("cuda:0"); m.reserve(8, "cuda:0")
    x = torch.from_numpy(make_crops(6, seed=29)).cuda()
    ref = None
    for v in [int(t) for t in "$VERS".split()]:
        m.set_option("stem_version", v)
        o = torch.empty(6, 112, 112, 32, dtype=torch.float16, device="cuda:0")
        _lib.check(lib.fac_debug_features_u8(m._ctx, x.data_ptr(), 6, 2, o.data_ptr(), None), m._ctx, "dbg")
        torch.cuda.synchronize()
        o = o.cpu()
        if ref is None: ref = o
        print(dt, v, "equal" if torch.equal(o, ref) else "DIFF", flush=True)
        assert torch.equal(o, ref)
    m._release()
PY
tail -3 gpurun_out/r03_stemab_eq.log
for rep in 1 2; do
for v in $VERS; do
  timeout -k 10 200 python -u bench.py --steps 50 --warmup 10 --no-fp16-line --no-video --no-s3d --no-resvitkan --no-repbn8 --no-cpu-baseline --opt stem_version=$v > gpurun_out/r03_stemab_$v.log 2>&1 || { tail -5 gpurun_out/r03_stemab_$v.log; exit 1; }
  python -c "import json,sys; l=json.loads(open('gpurun_out/r03_stemab_$v.log').read().strip().splitlines()[-1]); print('v$v', l['value'], l['ms_per_step'], l['roofline']['launch_ms'], l['roofline']['launch_ms_sync_profile'], l['roofline']['frac'])"
done
done
