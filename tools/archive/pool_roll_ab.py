"""Event timing of S3D's branch-3 MaxPool3d(3, 1, 1) (model.py:84-342) at the
config-4 shapes (B clips: 8x14x14 with 192 / 256 channels, 4x7x7 with 480 /
512 / 528 / 832), maxpool3_s1 (pool_roll 0) against maxpool3_roll (1: all
frames per thread, k: k frames), outputs checked bit-equal (relu'd random
data: non-negative, so no signed zeros).  GPU box only.

    python tools/pool_roll_ab.py [--B 384] [--reps 20] [--dtype bf16]
"""
import argparse
import ctypes
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from fac_fake_amd import _lib, ops  # noqa: E402


def timed(fn, reps):
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        ts.append((e0, e1))
    torch.cuda.synchronize()
    return sorted(a.elapsed_time(b) for a, b in ts)[len(ts) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=384)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--arms", default="0,1,4,2")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    lib = _lib.load()
    h = ctypes.c_void_p()
    _lib.check(lib.fac_create(0, _lib.DTYPES[a.dtype], ctypes.byref(h)), None, "fac_create")
    arms = [int(v) for v in a.arms.split(",")]
    print(f"{'shape':24s} " + " ".join(f"{'roll' + str(v):>9s}" for v in arms) + "   HBM-floor us", flush=True)
    tot = {v: 0.0 for v in arms}
    for d, hw, c in ((8, 14, 192), (8, 14, 256), (4, 7, 480), (4, 7, 512), (4, 7, 512), (4, 7, 512), (4, 7, 528),
                     (2, 3, 832), (2, 3, 832)):
        x = torch.randn(a.B, d, hw, hw, c, device=dev).relu().to(ops.TORCH16[a.dtype])
        outs, us = {}, {}
        for v in arms:
            _lib.check(lib.fac_set_option(h, b"pool_roll", v), h, "fac_set_option")
            o = ops.pool(x, 3, 1, 1, "max")
            torch.cuda.synchronize()
            outs[v] = o
            us[v] = timed(lambda: ops.pool(x, 3, 1, 1, "max"), a.reps) * 1e3
            tot[v] += us[v]
        same = all(torch.equal(outs[arms[0]], outs[v]) for v in arms)
        floor = 2 * x.numel() * 2 / 8e12 * 1e6
        print(f"{d}x{hw}x{hw}x{c:<4d} {'eq' if same else 'DIFF':4s}      " + " ".join(f"{us[v]:9.1f}" for v in arms)
              + f"   {floor:6.1f}", flush=True)
        assert same
    print("total                         " + " ".join(f"{tot[v]:9.1f}" for v in arms), flush=True)
    # maxpool3_lds14 (pool_lds14 1) vs maxpool3_s1 (0) on the 14x14 maps
    print("14x14 maps: pool_lds14 0 / 1 (us), HBM floor", flush=True)
    for d, hw, c in ((8, 14, 192), (8, 14, 256), (3, 14, 64)):
        x = torch.randn(a.B, d, hw, hw, c, device=dev).relu().to(ops.TORCH16[a.dtype])
        outs, us = {}, {}
        for v in (0, 1):
            _lib.check(lib.fac_set_option(h, b"pool_lds14", v), h, "fac_set_option")
            outs[v] = ops.pool(x, 3, 1, 1, "max")
            torch.cuda.synchronize()
            us[v] = timed(lambda: ops.pool(x, 3, 1, 1, "max"), a.reps) * 1e3
        same = torch.equal(outs[0], outs[1])
        floor = 2 * x.numel() * 2 / 8e12 * 1e6
        print(f"{d}x{hw}x{hw}x{c:<4d} {'eq' if same else 'DIFF'} {us[0]:9.1f} {us[1]:9.1f}   {floor:6.1f}", flush=True)
        assert same
    _lib.check(lib.fac_set_option(h, b"pool_lds14", 0), h, "fac_set_option")
    # maxpool3_s1's output frames per thread on the 14x14 maps (pool3_zg; 0 = all)
    print("maxpool3_s1 frames per thread: pool3_zg 0 / 1 / 2 / 4 (us)", flush=True)
    for d, hw, c in ((8, 14, 192), (8, 14, 256)):
        x = torch.randn(a.B, d, hw, hw, c, device=dev).relu().to(ops.TORCH16[a.dtype])
        outs, us = {}, {}
        for v in (0, 1, 2, 4):
            _lib.check(lib.fac_set_option(h, b"pool3_zg", v), h, "fac_set_option")
            outs[v] = ops.pool(x, 3, 1, 1, "max")
            torch.cuda.synchronize()
            us[v] = timed(lambda: ops.pool(x, 3, 1, 1, "max"), a.reps) * 1e3
        same = all(torch.equal(outs[0], outs[v]) for v in outs)
        print(f"{d}x{hw}x{hw}x{c:<4d} {'eq' if same else 'DIFF'} " + " ".join(f"{us[v]:9.1f}" for v in (0, 1, 2, 4)), flush=True)
        assert same
    _lib.check(lib.fac_set_option(h, b"pool3_zg", 0), h, "fac_set_option")
    _lib.check(lib.fac_set_option(h, b"pool_lds14", 1), h, "fac_set_option")
    # the strided max pools of S3D's base (model.py:17-33): pool_nd (pool_win 0) vs pool_max_win (1)
    print("strided pools: pool_win 0 / 1 (us), HBM floor", flush=True)
    for d, hw, c, k, st, pd in ((8, 56, 64, (1, 3, 3), (1, 2, 2), (0, 1, 1)), (8, 28, 192, (1, 3, 3), (1, 2, 2), (0, 1, 1)),
                                (8, 14, 480, 3, 2, 1), (4, 7, 832, 2, 2, 0)):
        x = torch.randn(a.B, d, hw, hw, c, device=dev).relu().to(ops.TORCH16[a.dtype])
        outs, us = {}, {}
        for v in (0, 1):
            _lib.check(lib.fac_set_option(h, b"pool_win", v), h, "fac_set_option")
            outs[v] = ops.pool(x, k, st, pd, "max")
            torch.cuda.synchronize()
            us[v] = timed(lambda: ops.pool(x, k, st, pd, "max"), a.reps) * 1e3
        same = torch.equal(outs[0], outs[1])
        floor = (x.numel() + outs[0].numel()) * 2 / 8e12 * 1e6
        print(f"{d}x{hw}x{hw}x{c:<4d} k{k} {'eq' if same else 'DIFF'} {us[0]:9.1f} {us[1]:9.1f}   {floor:6.1f}", flush=True)
        assert same
    _lib.check(lib.fac_set_option(h, b"pool_win", 1), h, "fac_set_option")
    _lib.check(lib.fac_set_option(h, b"pool_roll", 1), h, "fac_set_option")
    lib.fac_destroy(h)


if __name__ == "__main__":
    main()
