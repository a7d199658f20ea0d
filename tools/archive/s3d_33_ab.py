"""Event timing of S3D's (1,3,3) spatial convs at their config-4 shapes (B
clips): conv.hip's halo kernel (fac_conv3x3, the default where a tile
exists) against fac_conv_nd's persistent implicit GEMM (convnd_pt, the
uniform-tap gather; cin % 64 == 0 only), outputs compared in 16-bit ulps.
GPU box only.

    python tools/s3d_33_ab.py [--B 384] [--reps 20]
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
    print(f"{'layer':28s} {'conv.hip':>9s} {'conv_nd':>9s}  max rel diff  MFMA-floor us", flush=True)
    for hw, ci, co in ((28, 64, 192), (14, 128, 192), (14, 128, 128), (14, 256, 256)):
        w = torch.randn(co, ci, 1, 3, 3, generator=g) * (2.0 / (ci * 9)) ** 0.5
        b = torch.randn(co, generator=g) * 0.1
        L = ops.ConvLayer(w, b, 1, (0, 1, 1), dtype=a.dtype, device=dev)
        x = torch.randn(a.B, 8, hw, hw, ci, device=dev).relu().to(ops.TORCH16[a.dtype])
        y33 = L(x)
        torch.cuda.synchronize()
        t33 = timed(lambda: L(x), a.reps) * 1e3
        w33 = L._w33
        L._w33 = None   # fac_conv_nd route
        ynd = L(x)
        torch.cuda.synchronize()
        tnd = timed(lambda: L(x), a.reps) * 1e3
        L._w33 = w33
        rel = ((y33.float() - ynd.float()).abs().max() / y33.float().abs().max()).item()
        fl = 2.0 * a.B * 8 * hw * hw * co * ci * 9 / 2.5e15 * 1e6
        print(f"1x3x3 {ci}->{co} @8x{hw:<3d}        {t33:9.1f} {tnd:9.1f}  {rel:.2e}   {fl:7.1f}", flush=True)


if __name__ == "__main__":
    main()
