"""Per-stage GPU times of one CViT forward (fac_profile_forward_u8: a hipEvent
between stages) for a few batch sizes, mean of 5 after one warm-up.  GPU box.
    python tools/stage_ms.py --batch 1 8 29 [--dtype bf16] [--opt key=value]
"""
import argparse
import ctypes
import sys
from pathlib import Path

import numpy as np
import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from fac_fake_amd import _lib  # noqa: E402
from fac_fake_amd.cvit import CViT  # noqa: E402
from fac_fake_amd.weights import make_crops, make_state_dict  # noqa: E402

NAMES = [f"conv{i}" for i in range(1, 18)] + ["patch", "tf", "head"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, nargs="+", default=[1, 8, 29])
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--opt", action="append", default=[])
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    m = CViT(dtype=a.dtype)
    m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in make_state_dict(0).items()})
    m.to(dev)
    m.reserve(max(a.batch), dev)
    for o in a.opt:
        k, v = o.split("=")
        m.set_option(k, int(v))
    lib = _lib.load()
    for n in a.batch:
        crops = torch.from_numpy(make_crops(n, seed=7)).to(dev)
        m.forward_u8(crops, pos_index=torch.arange(n) % 32)
        p = (torch.arange(n, device=dev, dtype=torch.int32) % 32)
        lg = torch.empty(n, 2, device=dev)
        st = (ctypes.c_float * 20)()
        acc = np.zeros(20)
        for r in range(6):
            _lib.check(lib.fac_profile_forward_u8(m._ctx, crops.data_ptr(), n, p.data_ptr(), lg.data_ptr(), st, 20,
                                                  torch.cuda.current_stream().cuda_stream), m._ctx, "prof")
            if r:
                acc += np.frombuffer(st, dtype=np.float32)
        acc /= 5
        print(f"B={n:3d} sum {acc.sum() * 1e3:7.1f} us: " +
              " ".join(f"{k}={v * 1e3:.1f}" for k, v in zip(NAMES, acc) if k not in ("conv2", "conv3")), flush=True)


if __name__ == "__main__":
    main()
