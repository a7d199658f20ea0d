"""Same-box vendor-GEMM ceiling for the conv layers' implicit-GEMM shapes
(VERDICT r05 item 1).  Measurement only: torch.matmul (hipBLASLt on this
image) on the dense GEMM each 3x3 conv equals at B = 256 crops
(M = B*H*W pixels, N = Cout, K = 9*Cin), fp16 and bf16, random data, both
operand layouts; never used by the product path.  GPU box only.

    python tools/gemm_ceiling.py [--B 256]
"""
import argparse
import json

import torch

PEAK = 2516.6  # dense bf16/fp16 TFLOP/s (256 CU x 2.4 GHz x 4096 FLOP/clk/CU)

# name, H, Cin, Cout (cvit.py:99-147)
SHAPES = [("conv4", 112, 32, 64), ("conv5", 112, 64, 64), ("conv7", 56, 64, 128), ("conv8", 56, 128, 128),
          ("conv10", 28, 128, 256), ("conv11", 28, 256, 256), ("conv14", 14, 256, 512), ("conv15", 14, 512, 512)]


def time_mm(a, b, reps=20):
    for _ in range(3):
        torch.matmul(a, b)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        torch.matmul(a, b)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=256)
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    out = {}
    for name, H, cin, cout in SHAPES:
        M, N, K = args.B * H * H, cout, 9 * cin
        fl = 2.0 * M * N * K
        row = {"M": M, "N": N, "K": K}
        for dt in (torch.float16, torch.bfloat16):
            a = torch.randn(M, K, device=dev).to(dt)
            best = None
            for layout in ("nn", "nt"):
                b = torch.randn(K, N, device=dev).to(dt) if layout == "nn" else torch.randn(N, K, device=dev).to(dt).t()
                us = time_mm(a, b)
                if best is None or us < best[0]:
                    best = (us, layout)
                del b
            tag = "fp16" if dt == torch.float16 else "bf16"
            row[tag] = {"us": round(best[0], 1), "layout": best[1], "frac": round(fl / best[0] / 1e6 / PEAK, 3)}
            del a
            torch.cuda.empty_cache()
        out[name] = row
        print(name, json.dumps(row), flush=True)
    # reference points: a square GEMM (what the library reaches on an easy
    # shape) and one conv tap as its own GEMM (K = Cin: the nine per-tap
    # GEMMs of an implicit conv, without the 9x im2col operand)
    for name, M, N, K in (("square8192", 8192, 8192, 8192), ("conv15_tap", args.B * 196, 512, 512),
                          ("conv11_tap", args.B * 784, 256, 256)):
        row = {"M": M, "N": N, "K": K}
        for dt in (torch.float16, torch.bfloat16):
            a = torch.randn(M, K, device=dev).to(dt)
            b = torch.randn(N, K, device=dev).to(dt).t()
            us = time_mm(a, b)
            tag = "fp16" if dt == torch.float16 else "bf16"
            row[tag] = {"us": round(us, 1), "frac": round(2.0 * M * N * K / us / 1e6 / PEAK, 3)}
            del a, b
        out[name] = row
        print(name, json.dumps(row), flush=True)
    print(json.dumps({"gemm_ceiling": out, "B": args.B, "device": torch.cuda.get_device_name(0)}), flush=True)


if __name__ == "__main__":
    main()
