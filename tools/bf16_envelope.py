"""bf16 rounding envelope of every end-to-end golden fixture (VERDICT r03
item 1): max|dp| of the per-logit sigmoid between the oracle's emulation of
the HIP path's bf16 rounding points (fp32 accumulation, every operand and
stored activation rounded to bf16) and the reference module's fp32 golden,
on the fixture's own inputs.  The GPU tests gate bf16 at 1.25x these values
(instead of a flat 1e-2), so a bf16-only regression cannot hide in slack.

Test infrastructure only (imports oracle/).  Writes
tests/golden/bf16_envelope.json.

    python tools/bf16_envelope.py
"""
from __future__ import annotations

import json
import sys
from pathlib import Path

import numpy as np
import torch

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))

from fac_fake_amd.weights import (make_crops, make_resvitkan_state_dict, make_s3d_state_dict,  # noqa: E402
                                  make_state_dict, s3d_clips)
from oracle import cvit_torch, resvitkan_torch, s3d_torch  # noqa: E402

G = REPO / "tests" / "golden"


def _sig(x):
    return 1.0 / (1.0 + np.exp(-np.asarray(x, np.float64)))


def _dp(got, ref_logits):
    return float(np.abs(_sig(got) - _sig(ref_logits)).max())


@torch.no_grad()
def cvit_envelopes(dtype: str) -> dict:
    sd = make_state_dict(0)
    out = {}
    cases = {"golden_c1.npz": (make_crops(1, seed=1), np.array([0])),
             "golden_b32.npz": (make_crops(32, seed=2), np.arange(32)),
             "golden_b256.npz": (make_crops(256, seed=3), np.arange(256) % 32)}
    real = np.load(G / "golden_real.npz", allow_pickle=False)
    cases["golden_real.npz"] = (real["crops"], np.array([0, 1]))
    for name, (crops, slots) in cases.items():
        g = np.load(G / name, allow_pickle=False)
        ref = g["logits"] if "logits" in g else np.log(g["probs"] / (1 - g["probs"]))
        got = []
        for lo in range(0, len(crops), 32):
            x = cvit_torch.normalize_u8(crops[lo:lo + 32])
            got.append(cvit_torch.forward_emulated(sd, x, torch.from_numpy(slots[lo:lo + 32].astype(np.int64)),
                                                   dtype=dtype).numpy())
        out[name] = _dp(np.concatenate(got), ref)
        print(dtype, name, out[name], flush=True)
    return out


@torch.no_grad()
def resvitkan_envelope(dtype: str) -> dict:
    g = np.load(G / "resvitkan_golden.npz", allow_pickle=False)
    sd = make_resvitkan_state_dict(0)
    crops = make_crops(4, seed=int(g["crop_seed"]))
    got = resvitkan_torch.forward_emulated(sd, cvit_torch.normalize_u8(crops), dtype=dtype).numpy()
    v = _dp(got, g["logits"])
    print(dtype, "resvitkan", v, flush=True)
    return {"resvitkan_golden.npz": v}


@torch.no_grad()
def s3d_envelope(dtype: str) -> dict:
    g = np.load(G / "s3d_golden.npz", allow_pickle=False)
    x = torch.from_numpy(s3d_clips(2, 16, 112, seed=int(g["clip_seed"]))).float()
    out = {}
    for srm in ("no", "yes"):
        sd = make_s3d_state_dict(0, 1, srm == "yes")
        got = s3d_torch.forward_emulated(sd, x, srm == "yes", dtype=dtype).numpy()
        out[f"s3d_golden.npz:{srm}"] = _dp(got, g[f"logits_{srm}"])
        print(dtype, "s3d", srm, out[f"s3d_golden.npz:{srm}"], flush=True)
    return out


def main():
    torch.set_num_threads(8)
    env = {}
    for dt in ("bf16", "fp16"):
        e = {}
        e.update(cvit_envelopes(dt))
        e.update(resvitkan_envelope(dt))
        e.update(s3d_envelope(dt))
        env[dt] = {k: float(f"{v:.4g}") for k, v in e.items()}
    env["note"] = ("max|dp| of the oracle's emulated HIP rounding (oracle/*_torch.py forward_emulated) vs the fp32 "
                   "golden logits, per fixture; tools/bf16_envelope.py")
    (G / "bf16_envelope.json").write_text(json.dumps(env, indent=1, sort_keys=True) + "\n")


if __name__ == "__main__":
    main()
