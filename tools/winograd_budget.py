"""Winograd F(2x2, 3x3) error budget for the CViT conv stack.

Before any Winograd kernel is written for the MFMA-bound 28^2 / 14^2 layers
(cvit.py:110-147, conv10..conv17), this emulates what such a kernel would
round and reports max|dp| of the per-logit sigmoid against the fp32
reference module's outputs on golden_b256's crops, next to the direct-conv
16-bit path (tools/bf16_budget.py's all-16-bit policy: 4.1e-4 fp16, 5.1e-3
bf16 on the 256 crops).

Per Winograd layer, the kernel's arithmetic (Lavin & Gray 2016, F(2x2,3x3)):
  * input tiles d (4x4, stride 2, from the layer's 16-bit input; zero padding)
    -> V = B^T d B, exact in fp32 (entries 0/+-1), then rounded to 16 bits
    (the MFMA's A operand);
  * folded fp32 weights g (3x3) -> U = G g G^T in fp64, rounded to 16 bits
    once at load time (the B operand);
  * M = sum_c U . V per (i, j) of the 16 transformed positions, fp32
    accumulation (the MFMA accumulator);
  * Y = A^T M A in fp32, + bias, ReLU, (2x2 max), rounded to 16 bits like
    the direct path's output.
Every other rounding point is the direct path's (oracle emulation).

Two forms: F(2x2,3x3) (2-D, this file's winograd_conv: 4/9 of the MFMAs)
and F(2,3) along x (oracle.cvit_torch.conv3x3_wino_f23: what wino.hip
computes, 2/3 of the MFMAs).

Test infrastructure only (imports oracle/).

    python tools/winograd_budget.py [--n 256] [--threads 8]
"""
from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

import numpy as np
import torch
import torch.nn.functional as F

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))

from fac_fake_amd.weights import make_crops, make_state_dict  # noqa: E402
from oracle.cvit_torch import (LN_EPS, POOL_AFTER, _pos_rows, conv3x3_wino_f23, fold_bn,  # noqa: E402
                               forward_emulated, forward_fp32, normalize_u8, round_to, stem_indices, to_torch_sd)

BT = torch.tensor([[1, 0, -1, 0], [0, 1, 1, 0], [0, -1, 1, 0], [0, 1, 0, -1]], dtype=torch.float64)
G = torch.tensor([[1, 0, 0], [0.5, 0.5, 0.5], [0.5, -0.5, 0.5], [0, 0, 1]], dtype=torch.float64)
AT = torch.tensor([[1, 1, 1, 0], [0, 1, -1, -1]], dtype=torch.float64)


def winograd_conv(h: torch.Tensor, w: torch.Tensor, b: torch.Tensor, dt: str, tdt: str) -> torch.Tensor:
    """3x3/1 pad-1 conv of 16-bit-valued h [B,C,H,W] (fp32 tensor) by fp32
    weights w [K,C,3,3] as F(2x2,3x3) with V and U rounded to `tdt`."""
    Bn, C, H, W = h.shape
    K = w.shape[0]
    hp = F.pad(h, (1, 1, 1, 1))
    # 4x4 tiles at stride 2: [B, C, H/2, W/2, 4, 4]
    d = hp.unfold(2, 4, 2).unfold(3, 4, 2)
    bt = BT.float()
    V = torch.einsum("ia,ncyxae,je->ncyxij", bt, d, bt)  # exact in fp32: +-1 sums of 16-bit values
    V = round_to(V, tdt)
    U = torch.einsum("ia,kcae,je->kcij", G, w.double(), G)
    U = round_to(U.float(), tdt)
    out = torch.empty(Bn, K, H, W)
    at = AT.float()
    for i0 in range(0, Bn, 16):   # bound the [B, K, H/2, W/2, 4, 4] intermediate
        M = torch.einsum("kcij,ncyxij->nkyxij", U, V[i0:i0 + 16])   # fp32 accumulation
        Y = torch.einsum("pi,nkyxij,qj->nkyxpq", at, M, at)         # [b, K, H/2, W/2, 2, 2]
        out[i0:i0 + 16] = Y.permute(0, 1, 2, 4, 3, 5).reshape(-1, K, H, W)
    return out + b.view(1, -1, 1, 1)


@torch.no_grad()
def forward(sd, img, pos_index, dt: str, wino: set, tdt: str):
    """The oracle's 16-bit emulation of the HIP forward (every rounding
    point in `dt`), with the conv layers in `wino` (0-based) as Winograd."""
    sd = to_torch_sd(sd)
    r = lambda t: round_to(t, dt)  # noqa: E731
    h = r(img.float())
    for i, (ci, bi) in enumerate(stem_indices()):
        w, b = fold_bn(sd, ci, bi)
        if i in wino:
            h = F.relu(winograd_conv(h, w, b, dt, tdt))
        else:
            h = F.relu(F.conv2d(h, r(w), b, padding=1))
        if i in POOL_AFTER:
            h = F.max_pool2d(h, 2, 2)
        h = r(h)
    B = h.shape[0]
    y = h.permute(0, 2, 3, 1).reshape(B, 1, -1)
    y = F.linear(y, r(sd["patch_to_embedding.weight"]), sd["patch_to_embedding.bias"])
    x = torch.cat((sd["cls_token"].expand(B, -1, -1), y), 1) + _pos_rows(sd, pos_index, B)
    dim, heads, n = 1024, 8, 2
    for l in range(6):
        p = f"transformer.layers.{l}."
        hh = F.layer_norm(x, (dim,), sd[p + "0.fn.norm.weight"], sd[p + "0.fn.norm.bias"], LN_EPS)
        qkv = F.linear(r(hh), r(sd[p + "0.fn.fn.to_qkv.weight"]))
        q, k, v = qkv.view(B, n, 3, heads, dim // heads).permute(2, 0, 3, 1, 4)
        att = (torch.einsum("bhid,bhjd->bhij", q, k) * dim ** -0.5).softmax(dim=-1)
        o = torch.einsum("bhij,bhjd->bhid", att, v).permute(0, 2, 1, 3).reshape(B, n, dim)
        x = F.linear(r(o), r(sd[p + "0.fn.fn.to_out.weight"]), sd[p + "0.fn.fn.to_out.bias"]) + x
        hh = F.layer_norm(x, (dim,), sd[p + "1.fn.norm.weight"], sd[p + "1.fn.norm.bias"], LN_EPS)
        hh = F.gelu(F.linear(r(hh), r(sd[p + "1.fn.fn.net.0.weight"]), sd[p + "1.fn.fn.net.0.bias"]))
        x = F.linear(r(hh), r(sd[p + "1.fn.fn.net.2.weight"]), sd[p + "1.fn.fn.net.2.bias"]) + x
    c = r(x[:, 0])
    hh = F.relu(F.linear(c, r(sd["mlp_head.0.weight"]), sd["mlp_head.0.bias"]))
    return F.linear(hh, sd["mlp_head.2.weight"], sd["mlp_head.2.bias"])


def dp(a, b):
    return float((torch.sigmoid(a) - torch.sigmoid(b)).abs().max())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=256, help="crops of golden_b256's seed-3 batch")
    ap.add_argument("--threads", type=int, default=8)
    ap.add_argument("--out", default=None, help="write the table as JSON here")
    args = ap.parse_args()
    torch.set_num_threads(args.threads)
    sd = make_state_dict(0)
    crops = make_crops(256, seed=3)[: args.n]
    img = normalize_u8(crops)
    pos = np.arange(args.n) % 32
    ref = forward_fp32(sd, img, pos)
    rows = {}
    sets = {
        "direct (no Winograd)": set(),
        "conv14-17 (14^2)": set(range(13, 17)),
        "conv10-13 (28^2)": set(range(9, 13)),
        "conv10-17 (28^2 + 14^2)": set(range(9, 17)),
        "conv7-17 (56^2 and below)": set(range(6, 17)),
        "conv4-17 (112^2 and below)": set(range(3, 17)),
    }
    for dt in ("fp16", "bf16"):
        for name, s in sets.items():
            # F(2,3) along x: what conv3x3_wino (wino.hip) computes, via the oracle's emulation
            v = dp(forward_emulated(sd, img, pos, dt, wino=s), ref)
            rows[f"{dt}: F(2,3) x: {name}"] = v
            print(f"{dt}  F(2,3) along x   {name:28s} max|dp| {v:.3e}", flush=True)
            if s:
                v = dp(forward(sd, img, pos, dt, s, dt), ref)
                rows[f"{dt}: F(2x2,3x3): {name}"] = v
                print(f"{dt}  F(2x2,3x3)       {name:28s} max|dp| {v:.3e}", flush=True)
    if args.out:
        Path(args.out).write_text(json.dumps({"n_crops": args.n, "vs": "fp32 reference forward (oracle)",
                                              "bar": 1e-3, "max_abs_dprob": rows}, indent=1) + "\n")


if __name__ == "__main__":
    main()
