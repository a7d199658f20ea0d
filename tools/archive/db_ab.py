"""Same-process A/B of the conv3x3 kernel variants (fac_set_option "conv_db"):
bit-equality of every layer's output against the default kernel, then the
per-layer time of each arm (hipGraph of 20 launches, arms alternated).
GPU box only.

    python tools/db_ab.py [--dtype bf16] [--B 256] [--arms 0,7] [--reps 3]
"""
import argparse
import json
import sys
from pathlib import Path

import numpy as np
import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from fac_fake_amd import _lib  # noqa: E402
from fac_fake_amd.cvit import CViT  # noqa: E402
from fac_fake_amd.weights import make_state_dict  # noqa: E402
from tools.conv_sweep import LAYERS  # noqa: E402


PACKING_KEYS = ()   # options that change the weight packing (none left): one model per arm


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--B", type=int, default=256)
    ap.add_argument("--layers", default="4,5,6,7,8,9,10,11,12,13,14,15,16")
    ap.add_argument("--arms", default="0,7")
    ap.add_argument("--key", default="conv_db")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--pre", action="append", default=[], metavar="KEY=VALUE",
                    help="process-wide fac_set_option applied once before the arms (e.g. conv28_lds=32768)")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    arms = [int(a) for a in args.arms.split(",")]
    sd = {k: torch.from_numpy(np.asarray(v)) for k, v in make_state_dict(0).items()}
    # options that change the weight packing need one model per arm, packed
    # while that arm's value is set (the first arm must be the default); the
    # others share one model
    models = {}
    for a in (arms if args.key in PACKING_KEYS else arms[:1]):
        m = CViT(dtype=args.dtype)
        m.load_state_dict(sd)
        m.to(dev)
        if models:
            next(iter(models.values())).set_option(args.key, a)
        m.reserve(8, dev)
        models[a] = m
    model_of = (lambda a: models[a]) if args.key in PACKING_KEYS else (lambda a: models[arms[0]])
    for kv in args.pre:
        k, v = kv.split("=")
        model_of(arms[0]).set_option(k, int(v))
    lib = _lib.load()
    B = args.B
    res = {}
    tot = {a: 0.0 for a in arms}
    for layer in [int(x) for x in args.layers.split(",")]:
        H, Cin, Cout, pool = LAYERS[layer]
        g = torch.Generator(device="cpu").manual_seed(layer)
        x = (torch.rand(B, H, H, Cin, generator=g) * 2).to(
            torch.bfloat16 if args.dtype == "bf16" else torch.float16).to(dev)
        Ho = H // 2 if pool else H
        s = torch.cuda.Stream()
        outs, graphs = {}, {}
        for a in arms:
            m = model_of(a)
            m.set_option(args.key, a)
            y = torch.empty(B, Ho, Ho, Cout, dtype=x.dtype, device=dev)

            def call(y=y, m=m):
                _lib.check(lib.fac_debug_conv(m._ctx, layer, x.data_ptr(), B, y.data_ptr(),
                                              torch.cuda.current_stream().cuda_stream), m._ctx, "debug_conv")
            with torch.cuda.stream(s):
                call()
                torch.cuda.synchronize()
                gr = torch.cuda.CUDAGraph()
                with torch.cuda.graph(gr, stream=s):
                    for _ in range(20):
                        call()
            outs[a] = y
            graphs[a] = gr
        torch.cuda.synchronize()
        ref = outs[arms[0]].view(torch.int16)
        eq = {a: bool(torch.equal(outs[a].view(torch.int16), ref)) for a in arms}
        ndiff = {a: int((outs[a].view(torch.int16) != ref).sum()) for a in arms}
        times = {a: [] for a in arms}
        for _ in range(args.reps):
            for a in arms:
                model_of(a).set_option(args.key, a)
                graphs[a].replay()
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(3):
                    graphs[a].replay()
                e1.record()
                torch.cuda.synchronize()
                times[a].append(e0.elapsed_time(e1) * 1e3 / 60)
        fl = 2.0 * 9 * H * H * Cin * Cout * B
        row = {}
        for a in arms:
            us = min(times[a])
            tot[a] += us
            row[a] = {"us": round(us, 1), "frac": round(fl / us / 1e6 / 2516.6, 3), "bit_equal": eq[a],
                      "ndiff": ndiff[a]}
        res[f"conv{layer + 1}"] = row
        print(json.dumps({f"conv{layer + 1}": row}), flush=True)
    model_of(arms[0]).set_option(args.key, arms[0])
    print(json.dumps({"dtype": args.dtype, "total_us": {a: round(t, 1) for a, t in tot.items()}}), flush=True)


if __name__ == "__main__":
    main()
