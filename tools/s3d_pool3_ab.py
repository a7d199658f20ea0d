"""Same-process A/B of S3D's branch3 MaxPool3d(3,1,1) + 1x1x1 conv: fused
(FAC_CONV_MAXPOOL3S1, ops.hip maxpool3_pw) against fac_pool_nd then the conv
(`S3D.fuse_pool3 = False`).  One hipGraph per arm over the same model and
uint8 clips, replays alternated; prints ms per forward and the arms' max
logit difference.  GPU box only.

    python tools/s3d_pool3_ab.py [--B 1536] [--dtype bf16] [--rounds 3]
"""
import argparse
import sys
import time
from pathlib import Path

import numpy as np
import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from fac_fake_amd.s3d import S3D  # noqa: E402
from fac_fake_amd.weights import make_s3d_state_dict, s3d_clips  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=1536)
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--attr", default="fuse_pool3", choices=["fuse_pool3", "fuse_pool1", "fuse_sep"],
                    help="the S3D switch the arms toggle (branch3's pool, or base.1's)")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    m = S3D(1, "no", dtype=a.dtype)
    m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in make_s3d_state_dict(0, 1, False).items()})
    x = torch.from_numpy(s3d_clips(a.B, 16, 112, seed=50)).to(torch.uint8).to(dev)
    s = torch.cuda.Stream(dev)
    s.wait_stream(torch.cuda.current_stream(dev))
    graphs, outs = {}, {}
    with torch.cuda.stream(s):
        for arm in (True, False):
            setattr(m, a.attr, arm)
            m(x)
            torch.cuda.synchronize(dev)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=s):
                outs[arm] = m(x)
            graphs[arm] = g
        for g in graphs.values():
            g.replay()
        torch.cuda.synchronize(dev)
        d = (outs[True].float() - outs[False].float()).abs().max().item()
        print(f"{a.attr} B={a.B} {a.dtype}: max |logit fused - unfused| = {d:.3e}", flush=True)
        for r in range(a.rounds):
            for arm in (True, False):
                g = graphs[arm]
                g.replay()
                torch.cuda.synchronize(dev)
                t0 = time.perf_counter()
                for _ in range(a.steps):
                    g.replay()
                torch.cuda.synchronize(dev)
                ms = (time.perf_counter() - t0) / a.steps * 1e3
                print(f"round {r} {'fused  ' if arm else 'unfused'} {ms:8.3f} ms/forward  {a.B / ms * 1e3:9.1f} clips/s",
                      flush=True)


if __name__ == "__main__":
    main()
