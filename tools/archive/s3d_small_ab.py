"""Event timing of S3D's small-channel SepConv chains at 14x14 (Mixed_3b /
Mixed_3c branch2: (1,3,3) then (3,1,1), model.py:84-342), which run on the
per-lane tap gather of convnd_igemm (cin 16 / 32 / 96), against channel-padded
variants that take the uniform-tap gather (zero input channels / zero middle
channels, as the late blocks below 14x14 already do).  Random data, B clips of
8 frames; median of R back-to-back runs per chain.  GPU box only.

    python tools/s3d_small_ab.py [--B 384] [--reps 20]
"""
import argparse
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from fac_fake_amd import ops  # noqa: E402


def timed(fn, reps):
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        ts.append((e0, e1))
    torch.cuda.synchronize()
    return sorted(a.elapsed_time(b) for a, b in ts)[len(ts) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=384)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--dtype", default="bf16")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    g = torch.Generator().manual_seed(0)
    t16 = ops.TORCH16[a.dtype]

    def mk(co, ci, k, pad, cin_pad=None, cout_pad=None):
        w = torch.randn(co, ci, *k, generator=g) * (2.0 / (ci * k[0] * k[1] * k[2])) ** 0.5
        b = torch.randn(co, generator=g) * 0.1
        if cout_pad:
            w = torch.cat([w, torch.zeros(cout_pad - co, *w.shape[1:])])
            b = torch.cat([b, torch.zeros(cout_pad - co)])
        return ops.ConvLayer(w, b, 1, pad, dtype=a.dtype, device=dev, cin_pad=cin_pad)

    from fac_fake_amd import _lib
    import ctypes
    lib = _lib.load()
    h = ctypes.c_void_p()
    _lib.check(lib.fac_create(0, _lib.DTYPES[a.dtype], ctypes.byref(h)), None, "fac_create")

    def opt(v):
        _lib.check(lib.fac_set_option(h, b"nd_pt_wide", v), h, "fac_set_option")

    S, T = (1, 3, 3), (3, 1, 1)
    PS, PT = (0, 1, 1), (1, 0, 0)
    print(f"{'chain':44s} {'s us':>8s} {'t us':>8s} {'sum':>8s}", flush=True)
    for (ci, cm, co) in ((16, 32, 32), (32, 96, 96)):
        for name, cip, cmp_ in (("as run", None, None), ("mid pad 64", None, (cm + 63) // 64 * 64),
                                ("in+mid pad 64", (ci + 63) // 64 * 64, (cm + 63) // 64 * 64)):
            s = mk(cm, ci, S, PS, cin_pad=cip, cout_pad=cmp_)
            t = mk(co, cm, T, PT, cin_pad=cmp_)
            x = torch.randn(a.B, 8, 14, 14, s.cin_p, device=dev).to(t16)
            if cip:
                x[..., ci:] = 0
            mid = torch.empty(a.B, 8, 14, 14, s.cout if not cmp_ else cmp_, device=dev, dtype=t16)
            out = torch.empty(a.B, 8, 14, 14, co, device=dev, dtype=t16)
            fs = lambda: s(x, out=mid)  # noqa: E731
            ft = lambda: t(mid, out=out)  # noqa: E731
            res = {}
            for v in (0, 1024):
                opt(v)
                fs()
                ft()
                torch.cuda.synchronize()
                res[v] = out.float().clone()
                us_s, us_t = timed(fs, a.reps) * 1e3, timed(ft, a.reps) * 1e3
                print(f"{ci}->{cm}->{co} {name:22s} pt{v:<5d} {us_s:8.1f} {us_t:8.1f} {us_s + us_t:8.1f}", flush=True)
            print(f"    pt vs igemm max|d| {(res[0] - res[1024]).abs().max().item():.3g}", flush=True)
    # 1x1x1 branch-3 convs at 14x14 (cout 32 / 64): the new partial-block route
    for ci, co in ((192, 32), (256, 64)):
        L = mk(co, ci, (1, 1, 1), 0)
        x = torch.randn(a.B, 8, 14, 14, ci, device=dev).to(t16)
        out = torch.empty(a.B, 8, 14, 14, co, device=dev, dtype=t16)
        res = {}
        for v in (0, 1024):
            opt(v)
            L(x, out=out)
            torch.cuda.synchronize()
            res[v] = out.float().clone()
            us = timed(lambda: L(x, out=out), a.reps) * 1e3
            print(f"1x1 {ci}->{co} pt{v:<5d} {us:8.1f}", flush=True)
        print(f"    pt vs igemm max|d| {(res[0] - res[1024]).abs().max().item():.3g}", flush=True)


if __name__ == "__main__":
    main()
