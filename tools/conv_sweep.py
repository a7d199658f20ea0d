"""Time each stem conv kernel (fac_debug_conv, layers 1..16 = conv2..conv17)
in isolation at B crops, hipGraph of 20 launches.  GPU box only.

    python tools/conv_sweep.py [--dtype bf16] [--B 256] [--layers 3,4,...]
"""
import argparse
import json
import os
import sys
from pathlib import Path

import numpy as np
import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from fac_fake_amd import _lib  # noqa: E402
from fac_fake_amd.cvit import CViT  # noqa: E402
from fac_fake_amd.weights import make_state_dict  # noqa: E402

# (H, Cin, Cout, pool) of conv1..conv17 (cvit.py:86-148)
LAYERS = [(224, 3, 32, 0), (224, 32, 32, 0), (224, 32, 32, 1), (112, 32, 64, 0), (112, 64, 64, 0), (112, 64, 64, 1),
          (56, 64, 128, 0), (56, 128, 128, 0), (56, 128, 128, 1), (28, 128, 256, 0), (28, 256, 256, 0),
          (28, 256, 256, 0), (28, 256, 256, 1), (14, 256, 512, 0), (14, 512, 512, 0), (14, 512, 512, 0),
          (14, 512, 512, 1)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--B", type=int, default=256)
    ap.add_argument("--layers", default="3,4,5,6,7,8,9,10,11,12,13,14,15,16")
    ap.add_argument("--tag", default="")
    ap.add_argument("--opt", action="append", default=[], metavar="KEY=VALUE")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    m = CViT(dtype=args.dtype)
    m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in make_state_dict(0).items()})
    m.to(dev)
    m.reserve(8, dev)
    for kv in args.opt:
        k, v = kv.split("=")
        m.set_option(k, int(v))
    lib = _lib.load()
    B = args.B
    total = 0.0
    out = {}
    for layer in [int(x) for x in args.layers.split(",")]:
        H, Cin, Cout, pool = LAYERS[layer]
        x = (torch.rand(B, H, H, Cin, device=dev) * 2).to(torch.bfloat16 if args.dtype == "bf16" else torch.float16)
        Ho = H // 2 if pool else H
        y = torch.empty(B, Ho, Ho, Cout, dtype=x.dtype, device=dev)
        s = torch.cuda.Stream()

        def call():
            _lib.check(lib.fac_debug_conv(m._ctx, layer, x.data_ptr(), B, y.data_ptr(),
                                          torch.cuda.current_stream().cuda_stream), m._ctx, "debug_conv")
        with torch.cuda.stream(s):
            call()
            torch.cuda.synchronize()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=s):
                for _ in range(20):
                    call()
        g.replay()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(3):
            g.replay()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / 60
        fl = 2.0 * 9 * H * H * Cin * Cout * B
        total += us
        out[f"conv{layer + 1}"] = (round(us, 1), round(fl / us / 1e6 / 2516.6, 3))
    print(json.dumps({"tag": args.tag or ",".join(args.opt), "total_us": round(total, 1), "per_layer(us,frac)": out}), flush=True)


if __name__ == "__main__":
    main()
