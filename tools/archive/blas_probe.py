"""How fast the vendor GEMM (torch.matmul -> hipBLASLt on ROCm) runs ResNet-50's
non-residual 1x1 convs as plain [M, K] x [K, N] GEMMs (bias + ReLU in a
second op, so this is a lower bound on its time), next to the fac_conv_nd
launch of the same layer.  GPU box only:  python tools/blas_probe.py [B]
"""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from fac_fake_amd import ops  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
dev = torch.device("cuda:0")
SHAPES = [("512->128 @28", 28, 512, 128), ("512->256 @28", 28, 512, 256), ("1024->256 @14", 14, 1024, 256),
          ("1024->512 @14", 14, 1024, 512), ("2048->512 @7", 7, 2048, 512), ("256->64 @56", 56, 256, 64),
          ("128->512 @28", 28, 128, 512), ("256->1024 @14", 14, 256, 1024), ("512->2048 @7", 7, 512, 2048)]


def t_us(fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / reps


for name, h, k, n in SHAPES:
    m = B * h * h
    x = torch.randn(m, k, device=dev).to(torch.bfloat16)
    w = (torch.randn(n, k, device=dev) / k ** 0.5).to(torch.bfloat16)
    b = torch.randn(n, device=dev).to(torch.bfloat16)
    y = torch.empty(m, n, device=dev, dtype=torch.bfloat16)
    us_mm = t_us(lambda: torch.matmul(x, w.t(), out=y))
    us_lin = t_us(lambda: torch.nn.functional.linear(x, w, b))
    layer = ops.ConvLayer(torch.randn(n, k, 1, 1) / k ** 0.5, torch.randn(n), dtype="bf16", device=dev)
    xin = x.view(B, 1, h, h, k)
    us_fac = t_us(lambda: layer(xin, relu=True))
    byts = (m * k + m * n) * 2
    fl = 2.0 * m * n * k
    print(f"{name:14s} M={m:8d}  matmul {us_mm:7.1f} us ({byts / us_mm / 1e6:5.2f} TB/s, {fl / us_mm / 1e6:6.0f} TF/s)"
          f"  linear+bias {us_lin:7.1f}  fac_conv_nd {us_fac:7.1f} us", flush=True)
