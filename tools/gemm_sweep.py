"""Time every encoder GEMM call site (cvit_abi.hip forward_impl) in each tile
variant / split through fac_debug_gemm.  GPU box only:

    python tools/gemm_sweep.py [--dtype bf16] [--B 256]

Prints one line per (site, variant, splits): mean us per launch over a
hipGraph of 50 back-to-back launches (so launch gaps are the graph's).
"""
import argparse
import json
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from fac_fake_amd.cvit import CViT  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--B", type=int, default=256)
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    m = CViT(dtype=args.dtype)
    m.reserve(1, dev)
    tdt = torch.bfloat16 if args.dtype == "bf16" else torch.float16
    B, R = args.B, 2 * args.B
    sites = {  # name: (M, N, K, epi, splits options)
        "patch": (B, 1024, 25088, 4, [7, 14, 28]),
        "qkv": (R, 3072, 1024, 0, [1]),
        "out": (R, 1024, 1024, 4, [1, 2, 4]),
        "ff1": (R, 2048, 1024, 2, [1]),
        "ff2": (R, 1024, 2048, 4, [1, 2, 4]),
        "head": (B, 2048, 1024, 1, [1]),
    }
    res = []
    for name, (M, N, K, epi, splits) in sites.items():
        a = (torch.randn(M, K, device=dev) * 0.5).to(tdt)
        w = (torch.randn(N, K, device=dev) * 0.05).to(tdt)
        bias = torch.randn(N, device=dev)
        out = torch.empty(max(splits) * M * N, device=dev)
        for S in splits:
            for v in range(4):
                m.debug_gemm(epi, a, w, bias, out, splits=S, variant=v)
                torch.cuda.synchronize()
                g = torch.cuda.CUDAGraph()
                s = torch.cuda.Stream()
                with torch.cuda.stream(s):
                    with torch.cuda.graph(g, stream=s):
                        for _ in range(50):
                            m.debug_gemm(epi, a, w, bias, out, splits=S, variant=v)
                g.replay()
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(4):
                    g.replay()
                e1.record()
                torch.cuda.synchronize()
                us = e0.elapsed_time(e1) * 1e3 / 200
                tf = 2.0 * M * N * K / (us * 1e-6) / 1e12
                res.append({"site": name, "variant": v, "splits": S, "us": round(us, 2), "tflops": round(tf, 1)})
                print(json.dumps(res[-1]), flush=True)
    best = {}
    for r in res:
        if r["site"] not in best or r["us"] < best[r["site"]]["us"]:
            best[r["site"]] = r
    print("BEST", json.dumps(best))


if __name__ == "__main__":
    main()
