"""Same-box streaming ceiling for ResNet-50's bottleneck conv3 + residual
(relu(relu(conv1x1(x) + b) + res), ResVitKan.py:146-152) at config 5's
3072 crops: the fused 1x1 launch (ops.ConvLayer with residual, routed as in
the forward) against torch element-wise streams over the same bytes
(measurement only; torch is the yardstick, never the product path).

    python tools/res_ceiling.py [--B 3072] [--dtype bf16]
"""
import argparse
import sys
from pathlib import Path

import numpy as np
import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from fac_fake_amd.ops import ConvLayer  # noqa: E402


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
    for hw, cin, cout in ((28, 128, 512), (14, 256, 1024), (7, 512, 2048)):
        M = a.B * hw * hw
        x = torch.randn(a.B, 1, hw, hw, cin, device=dev).to(t16)
        r = torch.randn(a.B, 1, hw, hw, cout, device=dev).to(t16)
        o = torch.empty_like(r)
        w = torch.randn(cout, cin, 1, 1, 1) / np.sqrt(cin)
        layer = ConvLayer(w, torch.zeros(cout), 1, 0, dtype=a.dtype, device=dev)
        byts = 2.0 * M * (cin + 2 * cout)
        us = timed(lambda: layer(x, relu=True, out=o, residual=r, relu2=True))
        r2 = r.view(M, cout)
        o2 = o.view(M, cout)
        us_add = timed(lambda: torch.add(r2, o2, out=o2))          # 2 reads + 1 write of the M x cout map
        us_cp = timed(lambda: o2.copy_(r2))                          # 1 read + 1 write
        print(f"{cin}->{cout} @{hw}^2 M={M}: conv+res {us:8.1f} us {byts / us / 1e6:6.2f} TB/s | "
              f"torch add (3 x {2 * M * cout / 1e9:.2f} GB) {us_add:8.1f} us {6.0 * M * cout / us_add / 1e6:6.2f} TB/s | "
              f"copy {us_cp:8.1f} us {4.0 * M * cout / us_cp / 1e6:6.2f} TB/s", flush=True)


if __name__ == "__main__":
    main()
