"""Time ResNet-50's conv1 (+ maxpool) at config 5's batch: conv_s2d4, fac_pool_nd,
and the fused conv_s2d4_mp (FAC_CONV_MAXPOOL3S2), each over 20 back-to-back launches."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from fac_fake_amd.ops import ConvLayer, max_pool_sep

B = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
dev = "cuda:0"
g = torch.Generator().manual_seed(0)
layer = ConvLayer(torch.randn(64, 16, 1, 4, 4, generator=g) / 16, torch.randn(64, generator=g) * 0.1, 1, 0,
                  dtype="bf16", device=dev)
x = torch.randn(B, 1, 115, 115, 16, generator=g).to(torch.bfloat16).to(dev)
y = layer(x)


def t(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


conv = t(lambda: layer(x))
pool = t(lambda: max_pool_sep(y, (1, 3, 3), (1, 2, 2), (0, 1, 1)))
fused = t(lambda: layer(x, maxpool3s2=True))
mb_in, mb_c, mb_p = x.numel() * 2 / 1e6, y.numel() * 2 / 1e6, y.numel() / 2 / 1e6
fl = B * 112 * 112 * 64 * 256 * 2
print(f"B={B}: conv_s2d4 {conv:.1f} us, pool {pool:.1f} us, sum {conv + pool:.1f}; fused {fused:.1f} us "
      f"({(mb_in + mb_p) / fused:.2f} TB/s algorithmic, {fl / fused * 1e-6:.0f} TFLOP/s of the conv's FLOPs)")
