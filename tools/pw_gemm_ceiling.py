"""Same-box vendor-GEMM yardstick for ResNet-50's deep 1x1 convs at config
5's 3072 crops (ResVitKan.py:138-152): our 1x1 launch (ops.ConvLayer, routed
as in the forward: bias + ReLU epilogue, residual where the block has one)
against torch.matmul (hipBLASLt) of the same [M, K] x [K, N] GEMM without
any epilogue.  Measurement only: torch is the yardstick, never the product
path.

    python tools/pw_gemm_ceiling.py [--B 3072] [--dtype bf16]
"""
import argparse
import sys
from pathlib import Path

import numpy as np
import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from fac_fake_amd.ops import ConvLayer  # noqa: E402

# (map, cin, cout, residual): the K >= 512 1x1s and the layer4 conv3
SHAPES = ((14, 1024, 256, False), (14, 1024, 512, False), (7, 2048, 512, False), (7, 512, 2048, True),
          (28, 512, 256, False), (14, 256, 1024, True))


def timed(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e3  # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=3072)
    ap.add_argument("--dtype", default="bf16")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    t16 = torch.bfloat16 if a.dtype == "bf16" else torch.float16
    for hw, cin, cout, res in SHAPES:
        M = a.B * hw * hw
        x = torch.randn(a.B, 1, hw, hw, cin, device=dev).to(t16)
        o = torch.empty(a.B, 1, hw, hw, cout, device=dev, dtype=t16)
        r = torch.randn(a.B, 1, hw, hw, cout, device=dev).to(t16) if res else None
        w = torch.randn(cout, cin, 1, 1, 1) / np.sqrt(cin)
        layer = ConvLayer(w, torch.zeros(cout), 1, 0, dtype=a.dtype, device=dev)
        us = timed(lambda: layer(x, relu=True, out=o, residual=r, relu2=res))
        x2 = x.view(M, cin)
        wt = w.view(cout, cin).t().contiguous().to(t16).to(dev)
        o2 = o.view(M, cout)
        us_mm = timed(lambda: torch.matmul(x2, wt, out=o2))
        byts = 2.0 * M * (cin + cout * (2 if res else 1))
        fl = 2.0 * M * cin * cout
        print(f"{cin}->{cout}{' +res' if res else ''} @{hw}^2 M={M}: ours {us:8.1f} us {byts / us / 1e6:5.2f} TB/s "
              f"{fl / us / 1e6:6.1f} TF/s | torch.matmul (no epilogue) {us_mm:8.1f} us {fl / us_mm / 1e6:6.1f} TF/s",
              flush=True)


if __name__ == "__main__":
    main()
