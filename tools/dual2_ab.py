"""Same-process A/B of ResNet-50 layer2's first bottleneck end (conv3 128 ->
512 at 28^2 + the stride-2 downsample 256 -> 512 over the 56^2 block input):
pw_dual2 (fac_set_option "pw_res" 1) against the generic convnd_pt DUAL
route ("pw_res" 2), at config 5's 3072 crops.  Prints us per launch and the
achieved rate over the algorithmic bytes (h + the strided x rows + out, each
once).  GPU box only.

    python tools/dual2_ab.py [--n 3072] [--dtype bf16] [--rounds 3]
"""
import argparse
import ctypes
import sys
from pathlib import Path

import numpy as np
import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from fac_fake_amd import _lib  # noqa: E402
from fac_fake_amd.ops import ConvLayer, conv_dual  # noqa: E402

T16 = {"bf16": torch.bfloat16, "fp16": torch.float16}


def knob(v, dt):
    lib = _lib.load()
    h = ctypes.c_void_p()
    _lib.check(lib.fac_create(0, _lib.DTYPES[dt], ctypes.byref(h)), None, "fac_create")
    try:
        _lib.check(lib.fac_set_option(h, b"pw_res", v), h, "fac_set_option")
    finally:
        lib.fac_destroy(h)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=3072)
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--xstride", type=int, default=2, choices=[1, 2],
                    help="1: a compact 28^2 downsample input (measures the cost of the strided gather)")
    ap.add_argument("--layer", type=int, default=2, choices=[2, 3, 4],
                    help="3: layer3's pair (256 -> 1024 at 14^2, downsample 512 -> 1024 over 28^2)")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    dt = T16[a.dtype]
    g = torch.Generator().manual_seed(3)
    c3, hw = {2: (128, 28), 3: (256, 14), 4: (512, 7)}[a.layer]
    cds, cout = 2 * c3, 4 * c3
    l3 = ConvLayer(torch.randn(cout, c3, 1, 1, 1, generator=g) / np.sqrt(c3), torch.randn(cout, generator=g) * 0.1,
                   1, 0, dtype=a.dtype, device=dev)
    ld = ConvLayer(torch.randn(cout, cds, 1, 1, 1, generator=g) / np.sqrt(cds), torch.randn(cout, generator=g) * 0.1,
                   (1, a.xstride, a.xstride), 0, dtype=a.dtype, device=dev)
    h = torch.randn(a.n, 1, hw, hw, c3, device=dev).to(dt)
    x = torch.randn(a.n, 1, hw * a.xstride, hw * a.xstride, cds, device=dev).to(dt)
    out = torch.empty(a.n, 1, hw, hw, cout, device=dev, dtype=dt)
    M = a.n * hw * hw
    nbytes = M * (c3 + cds + cout) * 2
    res = {}
    try:
        for v in (1, 2):
            knob(v, a.dtype)
            conv_dual(l3, h, ld, x, out=out)
            torch.cuda.synchronize()
            res[v] = out.clone()
        d = (res[1].float() - res[2].float()).abs().max().item()
        print(f"layer{a.layer} dual n={a.n} {a.dtype} x stride {a.xstride}: M={M}, algorithmic {nbytes / 1e9:.3f} GB; "
              f"max |pw_dual2 - convnd_pt| = {d:.3e}", flush=True)
        for r in range(a.rounds):
            for v in (1, 2):
                knob(v, a.dtype)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                conv_dual(l3, h, ld, x, out=out)
                e0.record()
                for _ in range(a.iters):
                    conv_dual(l3, h, ld, x, out=out)
                e1.record()
                torch.cuda.synchronize()
                us = e0.elapsed_time(e1) / a.iters * 1e3
                print(f"round {r} {'pw_dual2 ' if v == 1 else 'convnd_pt'} {us:9.1f} us  "
                      f"{nbytes / us / 1e6:6.2f} TB/s", flush=True)
    finally:
        knob(1, a.dtype)


if __name__ == "__main__":
    main()
