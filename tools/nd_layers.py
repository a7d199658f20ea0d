"""Event timing of single fac_conv_nd layers at the ResVitKan (ResNet-50, B
crops) shapes that still run on convnd_igemm, on random data: each layer R
times back to back (median), with its algorithmic TFLOP/s, its minimum HBM
GB/s (input pixels the conv reads once + output (+ residual)), and for the
stride-1 1x1 layers torch.matmul (hipBLASLt) on the same GEMM as a library
comparison.  `--only i` runs layer i alone (for rocprofv3 --pmc passes).
GPU box only.

    python tools/nd_layers.py [--B 512] [--reps 10] [--only i] [--no-torch]
"""
import argparse
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from fac_fake_amd import ops  # noqa: E402

# (h_in, cin, cout, k, stride, pad, residual)
LAYERS = [
    (28, 512, 256, 1, 1, 0, False),
    (14, 1024, 512, 1, 1, 0, False),
    (56, 256, 512, 1, 2, 0, False),
    (28, 512, 1024, 1, 2, 0, False),
    (14, 1024, 2048, 1, 2, 0, False),
    (56, 128, 128, 3, 2, 1, False),
    (28, 256, 256, 3, 2, 1, False),
    (14, 512, 512, 3, 2, 1, False),
    (7, 512, 512, 3, 1, 1, False),
    (7, 512, 2048, 1, 1, 0, True),
    (7, 2048, 512, 1, 1, 0, False),
    (14, 1024, 256, 1, 1, 0, False),
    (28, 512, 128, 1, 1, 0, False),
]


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
    ap.add_argument("--B", type=int, default=512)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--only", type=int, default=-1)
    ap.add_argument("--no-torch", action="store_true")
    ap.add_argument("--dtype", default="bf16")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    g = torch.Generator().manual_seed(0)
    print(f"{'layer':30s} {'us':>8s} {'TF/s':>7s} {'GB/s':>6s} {'torch us':>9s}", flush=True)
    for i, (h, ci, co, k, s, p, res) in enumerate(LAYERS):
        if a.only >= 0 and i != a.only:
            continue
        w = torch.randn(co, ci, k, k, generator=g) * (2.0 / (ci * k * k)) ** 0.5
        b = torch.randn(co, generator=g) * 0.1
        layer = ops.ConvLayer(w, b, stride=s, padding=p, dtype=a.dtype, device=dev)
        x = torch.randn(a.B, 1, h, h, ci, device=dev).to(ops.TORCH16[a.dtype])
        ho = (h + 2 * p - k) // s + 1
        r = torch.randn(a.B, 1, ho, ho, co, device=dev).to(x.dtype) if res else None
        out = torch.empty(a.B, 1, ho, ho, co, device=dev, dtype=x.dtype)
        fn = lambda: layer(x, out=out, residual=r, relu2=res)  # noqa: E731
        fn()
        torch.cuda.synchronize()
        ms = timed(fn, a.reps)
        M = a.B * ho * ho
        fl = 2.0 * M * co * ci * k * k
        pix_in = a.B * (h * h if k > 1 or s == 1 else ho * ho)
        by = 2.0 * (pix_in * ci + M * co * (2 if res else 1))
        tms = ""
        if k == 1 and s == 1 and not a.no_torch:
            A = x.reshape(M, ci)
            Wt = layer.w[:co].reshape(co, -1)[:, :ci]
            A @ Wt.t()
            torch.cuda.synchronize()
            tms = f"{timed(lambda: A @ Wt.t(), a.reps) * 1e3:9.1f}"
        name = f"{k}x{k}/{s} {ci}->{co} @{h}{' +res' if res else ''}"
        print(f"{name:30s} {ms * 1e3:8.1f} {fl / ms / 1e9:7.1f} {by / ms / 1e6:6.0f} {tms}", flush=True)


if __name__ == "__main__":
    main()
