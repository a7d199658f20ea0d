"""A few eager S3D forwards (config 4: B raw 16x112x112 clips, SRM off) for
rocprofv3 --kernel-trace: every launch of one forward in order
(tools/trace_order.py lists the last forward's dispatches).  GPU box only.

    rocprofv3 --kernel-trace --output-format csv -d DIR -o run -- python3 tools/s3d_eager.py [--B 384]
"""
import argparse
import sys
from pathlib import Path

import numpy as np
import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from fac_fake_amd.s3d import S3D  # noqa: E402
from fac_fake_amd.weights import make_s3d_state_dict, s3d_clips  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=384)
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--u8", action="store_true", help="uint8 clips (decoded frames: base.0 as one launch)")
    ap.add_argument("--no-fuse", action="store_true", help="with --u8: base.0 as two launches")
    ap.add_argument("--no-pool3", action="store_true", help="branch3's MaxPool3d(3,1,1) as its own launch")
    ap.add_argument("--opt", action="append", default=[], help="process-wide fac_set_option knob, name=value")
    a = ap.parse_args()
    if a.opt:
        import ctypes
        from fac_fake_amd import _lib
        lib = _lib.load()
        h = ctypes.c_void_p()
        _lib.check(lib.fac_create(0, _lib.DTYPES[a.dtype], ctypes.byref(h)), None, "fac_create")
        for kv in a.opt:
            k, v = kv.split("=")
            _lib.check(lib.fac_set_option(h, k.encode(), int(v)), h, "fac_set_option")
        lib.fac_destroy(h)
    dev = torch.device("cuda:0")
    m = S3D(1, "no", dtype=a.dtype)
    m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in make_s3d_state_dict(0, 1, False).items()})
    clips = torch.from_numpy(s3d_clips(a.B, 16, 112, seed=3)).to(dev)
    if a.u8:
        clips = clips.to(torch.uint8)
    m.fuse_base0 = not a.no_fuse
    m.fuse_pool3 = not a.no_pool3
    for _ in range(a.reps):
        m(clips)
        torch.cuda.synchronize()
    print("done", flush=True)


if __name__ == "__main__":
    main()
