"""Kernel trace target for the reference's one-video call (B = 29 crops,
cvit_prediction.py:224-229): N eager forwards (graph_max_b 0, so every
kernel launch is its own record) after warm-up.  Run under
    rocprofv3 --kernel-trace --stats -d gpurun_out/prof_small -- python tools/small_b_trace.py
"""
import argparse
import sys
from pathlib import Path

import numpy as np
import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from fac_fake_amd.cvit import CViT  # noqa: E402
from fac_fake_amd.weights import make_state_dict  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--batch", type=int, default=29)
    ap.add_argument("--reps", type=int, default=300)
    ap.add_argument("--warmup", type=int, default=200)
    ap.add_argument("--graph", action="store_true")
    ap.add_argument("--opt", action="append", default=[])
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    m = CViT(dtype=args.dtype)
    m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in make_state_dict(0).items()})
    m.to(dev)
    m.reserve(256, dev)
    if not args.graph:
        m.set_option("graph_max_b", 0)
    for o in args.opt:
        k, v = o.split("=")
        m.set_option(k, int(v))
    g = torch.Generator().manual_seed(5)
    x = torch.randint(0, 256, (args.batch, 224, 224, 3), dtype=torch.uint8, generator=g).to(dev)
    for _ in range(args.warmup):  # clocks ramp up over ~0.1 s of work
        m.forward_u8(x)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(args.reps):
        m.forward_u8(x)
    e.record()
    torch.cuda.synchronize()
    print(f"B={args.batch} {args.dtype} {'graph' if args.graph else 'eager'}: {s.elapsed_time(e) / args.reps:.4f} ms/forward")


if __name__ == "__main__":
    main()
