"""Config-4 S3D forward (B raw 16x112x112 clips, one hipGraph per step) with
the clips resident as fp32 vs uint8 (fac_conv_s2d4_clip vs _u8), alternated
in one process; logits checked equal.  GPU box only.

    python tools/s3d_input_ab.py [--B 384] [--steps 20] [--rounds 3]
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
    ap.add_argument("--B", type=int, default=384)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    m = S3D(1, "no", dtype="bf16")
    m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in make_s3d_state_dict(0, 1, False).items()})
    x32 = torch.from_numpy(s3d_clips(a.B, 16, 112, seed=50)).to(dev)
    x8 = x32.to(torch.uint8)
    s = torch.cuda.Stream(dev)
    s.wait_stream(torch.cuda.current_stream(dev))
    graphs, outs = {}, {}
    with torch.cuda.stream(s):
        for name, x in (("f32", x32), ("u8", x8)):
            m(x)
            torch.cuda.synchronize(dev)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=s):
                outs[name] = m(x)
            graphs[name] = g
        for r in range(a.rounds):
            for name, g in graphs.items():
                for _ in range(3):
                    g.replay()
                torch.cuda.synchronize(dev)
                t0 = time.perf_counter()
                for _ in range(a.steps):
                    g.replay()
                torch.cuda.synchronize(dev)
                el = time.perf_counter() - t0
                print(f"round {r} {name:4s} {a.B * a.steps / el:9.1f} clips/s  {el / a.steps * 1e3:7.3f} ms", flush=True)
    print("logits equal:", torch.equal(outs["f32"], outs["u8"]), flush=True)


if __name__ == "__main__":
    main()
