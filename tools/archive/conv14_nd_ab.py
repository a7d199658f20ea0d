"""Same-box timing of one CViT-shaped 3x3 conv (B crops, HxH, cin -> cout,
bias + ReLU) on conv.hip's box kernel (fac_conv3x3) vs the generic implicit
GEMM of ops.hip (fac_conv_nd: convnd_pt / convnd_igemm), with the max
difference between the two outputs.
    python tools/conv14_nd_ab.py [--h 14 --cin 512 --cout 512 --batch 256]
"""
import argparse
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from fac_fake_amd import ops  # noqa: E402


def timed(f, reps=20):
    for _ in range(3):
        f()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        f()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--h", type=int, default=14)
    ap.add_argument("--cin", type=int, default=512)
    ap.add_argument("--cout", type=int, default=512)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--dtype", default="bf16")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    g = torch.Generator().manual_seed(0)
    w = torch.randn(a.cout, a.cin, 3, 3, generator=g) * (2.0 / (9 * a.cin)) ** 0.5
    b = torch.randn(a.cout, generator=g) * 0.1
    box = ops.ConvLayer(w, b, 1, 1, dtype=a.dtype, device=dev)
    nd = ops.ConvLayer(w, b, 1, 1, dtype=a.dtype, device=dev)
    nd._w33 = None
    x = (torch.randn(a.batch, 1, a.h, a.h, a.cin, generator=g)).to(ops.TORCH16[a.dtype]).to(dev)
    ob, on = box(x), nd(x)
    torch.cuda.synchronize()
    flop = 2.0 * a.batch * a.h * a.h * 9 * a.cin * a.cout
    tb, tn = timed(lambda: box(x, out=ob)), timed(lambda: nd(x, out=on))
    d = (ob.float() - on.float()).abs().max().item()
    print(f"{a.h}^2 {a.cin}->{a.cout} B={a.batch} {a.dtype}: box {tb:.1f} us ({flop / tb / 1e6:.0f} TF/s), "
          f"conv_nd {tn:.1f} us ({flop / tn / 1e6:.0f} TF/s), max|diff| {d:.3g}")


if __name__ == "__main__":
    main()
