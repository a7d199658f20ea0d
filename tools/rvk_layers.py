"""Per-layer timing of the fac_conv_nd launches of the ResVitKan ResNet-50 stem
(--model rvk, B crops) or of S3D (--model s3d, B 16x112x112 clips): each
layer's median event-timed duration over a few eager forwards, with its
algorithmic TFLOP/s and minimum HBM GB/s.  GPU box only.

    python tools/rvk_layers.py [--model rvk|s3d] [--B 256] [--dtype bf16] [--u8]
"""
import argparse
import sys
from collections import defaultdict
from pathlib import Path

import numpy as np
import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from fac_fake_amd import ops  # noqa: E402
from fac_fake_amd.resvitkan import ResVitKan  # noqa: E402
from fac_fake_amd.weights import make_crops, make_resvitkan_state_dict  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="rvk", choices=["rvk", "s3d"])
    ap.add_argument("--B", type=int, default=0)
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--u8", action="store_true", help="S3D: uint8 clips (decoded frames; base.0 as one launch)")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    if a.model == "rvk":
        a.B = a.B or 256
        m = ResVitKan(dtype=a.dtype)
        m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in make_resvitkan_state_dict(0).items()})
        crops = torch.from_numpy(make_crops(a.B, seed=3)).to(dev)
        pidx = torch.arange(a.B, dtype=torch.int32, device=dev) % 32
        run = lambda: m.forward_u8(crops, pos_index=pidx)  # noqa: E731
    else:
        from fac_fake_amd.s3d import S3D
        from fac_fake_amd.weights import make_s3d_state_dict, s3d_clips
        a.B = a.B or 64
        m = S3D(1, "no", dtype=a.dtype)
        m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in make_s3d_state_dict(0, 1, False).items()})
        clips = torch.from_numpy(s3d_clips(a.B, 16, 112, seed=3)).to(dev)
        if a.u8:
            clips = clips.to(torch.uint8)
        run = lambda: m(clips)  # noqa: E731
    run()
    torch.cuda.synchronize()
    rec = []
    orig = ops.ConvLayer.__call__

    def timed(self, x, **kw):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        out = orig(self, x, **kw)
        e1.record()
        n, d, h, w, c = x.shape
        od, oh, ow = self.out_dims(d, h, w)
        M = n * od * oh * ow
        K = self.g.kd * self.g.kh * self.g.kw * self.cin
        flops = 2.0 * M * self.cout * K
        byts = 2.0 * (n * d * h * w * c + M * self.cout * (2 if kw.get("residual") is not None else 1))
        rec.append((f"{self.g.kd}x{self.g.kh}x{self.g.kw}/{self.g.sd}{self.g.sh} {self.cin}->{self.cout} @{d}x{h}", M,
                    self.cout, K, flops,
                    byts, e0, e1))
        return out

    from fac_fake_amd import resvitkan as rvk_mod
    orig_dual = ops.conv_dual

    def timed_dual(layer, h, ds, x, **kw):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        out = orig_dual(layer, h, ds, x, **kw)
        e1.record()
        M = out.numel() // layer.cout
        K = layer.cin + ds.g.kh * ds.g.kw * ds.cin
        flops = 2.0 * M * layer.cout * K
        byts = 2.0 * (h.numel() + x.numel() + out.numel())
        rec.append((f"dual {layer.cin}+{ds.cin}/{ds.g.sh}->{layer.cout} @{h.shape[2]}", M, layer.cout, K, flops, byts,
                    e0, e1))
        return out

    ops.conv_dual = rvk_mod.conv_dual = timed_dual
    ops.ConvLayer.__call__ = timed
    acc = defaultdict(list)
    meta = {}
    for _ in range(a.reps):
        rec.clear()
        run()
        torch.cuda.synchronize()
        for i, (name, M, N, K, fl, by, e0, e1) in enumerate(rec):
            acc[i].append(e0.elapsed_time(e1))
            meta[i] = (name, M, N, K, fl, by)
    tot = 0.0
    print(f"{'layer':28s} {'M':>8s} {'N':>5s} {'K':>5s} {'us':>8s} {'TF/s':>7s} {'GB/s':>7s}")
    for i in sorted(acc):
        name, M, N, K, fl, by = meta[i]
        ms = float(np.median(acc[i]))
        tot += ms
        print(f"{name:28s} {M:8d} {N:5d} {K:5d} {ms * 1e3:8.1f} {fl / ms / 1e9:7.1f} {by / ms / 1e6:7.0f}")
    print(f"total conv ms {tot:.3f}")


if __name__ == "__main__":
    main()
