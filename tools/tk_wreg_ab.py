"""Same-process A/B of S3D's cin-192 (3,1,1) temporal convs (SepConv3d
conv_t, model.py:63-82) on conv_tk2 with the weights in VGPRs
(fac_set_option "tk_wreg" 1) or in LDS ("tk_wreg" 0), at config 4's 1536
clips: base.3's 192 -> 192 at 8 x 28^2 and Mixed_3c's branch1 192 -> 192 at
8 x 14^2.  Prints us per launch and the MFMA rate.  GPU box only.

    python tools/tk_wreg_ab.py [--n 1536] [--dtype bf16] [--rounds 3]
"""
import argparse
import ctypes
import sys
from pathlib import Path

import numpy as np
import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from fac_fake_amd import _lib  # noqa: E402
from fac_fake_amd.ops import ConvLayer  # noqa: E402

T16 = {"bf16": torch.bfloat16, "fp16": torch.float16}


def knob(v, dt):
    lib = _lib.load()
    h = ctypes.c_void_p()
    _lib.check(lib.fac_create(0, _lib.DTYPES[dt], ctypes.byref(h)), None, "fac_create")
    try:
        _lib.check(lib.fac_set_option(h, b"tk_wreg", v), h, "fac_set_option")
    finally:
        lib.fac_destroy(h)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1536)
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--cin", type=int, default=192, choices=[128, 192])
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    dt = T16[a.dtype]
    g = torch.Generator().manual_seed(3)
    c = a.cin
    layer = ConvLayer(torch.randn(c, c, 3, 1, 1, generator=g) / np.sqrt(3 * c), torch.randn(c, generator=g) * 0.1, 1,
                      (1, 0, 0), dtype=a.dtype, device=dev)
    try:
        for hw in ((28, 14) if c == 192 else (14,)):
            x = torch.randn(a.n, 8, hw, hw, c, device=dev).to(dt)
            out = torch.empty(a.n, 8, hw, hw, c, device=dev, dtype=dt)
            fl = 2.0 * a.n * 8 * hw * hw * c * 3 * c
            res = {}
            for v in (1, 0):
                knob(v, a.dtype)
                layer(x, relu=True, out=out)
                torch.cuda.synchronize()
                res[v] = out.clone()
            print(f"(3,1,1) {c}->{c} at {a.n} x 8 x {hw}^2 {a.dtype}: bit-identical {torch.equal(res[0], res[1])}",
                  flush=True)
            for r in range(a.rounds):
                for v in (1, 0):
                    knob(v, a.dtype)
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    layer(x, relu=True, out=out)
                    e0.record()
                    for _ in range(a.iters):
                        layer(x, relu=True, out=out)
                    e1.record()
                    torch.cuda.synchronize()
                    us = e0.elapsed_time(e1) / a.iters * 1e3
                    print(f"round {r} {'weights in VGPRs' if v else 'weights in LDS  '} {us:9.1f} us  "
                          f"{fl / us / 1e6:7.1f} TF/s", flush=True)
            del x, out
    finally:
        knob(1, a.dtype)


if __name__ == "__main__":
    main()
