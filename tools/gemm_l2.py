"""How much of a few-row encoder GEMM's time is its weight stream's source
(measurement only, GPU box): each call site at M = 2B rows (B = 29, the
reference's one-video call) timed in a hipGraph of 20 launches
  * hot:  back to back (its weights stay in the XCDs' L2 between launches);
  * cold: each launch behind a copy between two other buffers (--flush-mb:
          128 MB also evicts the Infinity Cache, so the weights come from
          HBM; 24 MB only the XCDs' L2s, so they come from the Infinity
          Cache, as in a loop of one-video forwards), minus the copies alone.
The difference bounds what staging the next GEMM's weights into L2 during
the previous (latency-bound) kernel could save per launch.

    python tools/gemm_l2.py [--dtype fp16] [--B 29]
"""
import argparse
import json
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from fac_fake_amd.cvit import CViT  # noqa: E402


def graph_us(fn, reps=20):
    s = torch.cuda.Stream()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        fn()
        torch.cuda.synchronize()
        with torch.cuda.graph(g, stream=s):
            for _ in range(reps):
                fn()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(3):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / (3 * reps)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dtype", default="fp16")
    ap.add_argument("--B", type=int, default=29)
    ap.add_argument("--flush-mb", type=int, default=128,
                    help="bytes copied between launches: 128 evicts L2 and the Infinity Cache, 24 only the L2s")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    m = CViT(dtype=args.dtype)
    m.reserve(1, dev)
    tdt = torch.bfloat16 if args.dtype == "bf16" else torch.float16
    B, R = args.B, 2 * args.B
    src = torch.empty(args.flush_mb << 19, dtype=torch.float16, device=dev)
    dst = torch.empty_like(src)
    sites = {"patch": (B, 1024, 25088, 4, 14), "qkv": (R, 3072, 1024, 0, 1), "out": (R, 1024, 1024, 4, 4),
             "ff1": (R, 2048, 1024, 2, 1), "ff2": (R, 1024, 2048, 4, 4), "head": (B, 2048, 1024, 1, 1)}
    flush = graph_us(lambda: dst.copy_(src))
    res = {"flush_us": round(flush, 1)}
    for name, (M, N, K, epi, S) in sites.items():
        a = (torch.randn(M, K, device=dev) * 0.5).to(tdt)
        w = (torch.randn(N, K, device=dev) * 0.05).to(tdt)
        bias = torch.randn(N, device=dev)
        out = torch.empty(S * M * N, device=dev)

        def gemm():
            m.debug_gemm(epi, a, w, bias, out, splits=S)

        def cold():
            dst.copy_(src)
            gemm()
        hot = graph_us(gemm)
        c = graph_us(cold) - flush
        res[name] = {"M": M, "N": N, "K": K, "weights_MB": round(N * K * 2 / 1e6, 2), "hot_us": round(hot, 2),
                     "cold_us": round(c, 2)}
        print(name, json.dumps(res[name]), flush=True)
    print(json.dumps({"gemm_l2": res, "B": B, "dtype": args.dtype, "flush_mb": args.flush_mb}), flush=True)


if __name__ == "__main__":
    main()
