"""bf16 error budget of the CViT forward.

Runs the oracle's emulation of the HIP path with a per-rounding-point policy
(fp32 = not rounded, bf16, fp16) and reports max|dp| of the per-logit sigmoid
against the fp32 reference on the golden crops.  Rounding points, in the
order the HIP path meets them:

  input        normalised conv1 input (LUT output)
  w_conv<i>    BN-folded weight of conv i (0-based)
  a_conv<i>    output of conv i after bias+ReLU(+pool)
  w_patch      patch-embedding weight [1024, 25088]
  w_tail       transformer + head weight matrices
  a_ln         LayerNorm outputs entering QKV / FF1
  a_attn       attention output entering to_out
  a_gelu       GELU output entering FF2
  a_cls        CLS rows entering the head

Test infrastructure only (imports oracle/).

  python tools/bf16_budget.py [--n 64]
"""
from __future__ import annotations

import argparse
import sys
from pathlib import Path

import numpy as np
import torch
import torch.nn.functional as F

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))

from fac_fake_amd.weights import make_crops, make_state_dict  # noqa: E402
from oracle.cvit_torch import (LN_EPS, POOL_AFTER, _pos_rows, fold_bn, forward_fp32, normalize_u8,  # noqa: E402
                               round_to, stem_indices, to_torch_sd)

POINTS = (["input"] + [f"w_conv{i}" for i in range(17)] + [f"a_conv{i}" for i in range(17)]
          + ["w_patch", "w_tail", "a_ln", "a_attn", "a_gelu", "a_cls"])


def _r(policy, name):
    d = policy.get(name, "fp32")
    if d == "fp32":
        return lambda t: t
    return lambda t: round_to(t, d)


@torch.no_grad()
def forward_policy(sd, img, pos_index, policy):
    sd = to_torch_sd(sd)
    h = _r(policy, "input")(img.float())
    for i, (ci, bi) in enumerate(stem_indices()):
        w, b = fold_bn(sd, ci, bi)
        h = F.relu(F.conv2d(h, _r(policy, f"w_conv{i}")(w), b, padding=1))
        if i in POOL_AFTER:
            h = F.max_pool2d(h, 2, 2)
        h = _r(policy, f"a_conv{i}")(h)
    B = h.shape[0]
    rw, rp = _r(policy, "w_tail"), _r(policy, "w_patch")
    ln, at, ge, cl = (_r(policy, k) for k in ("a_ln", "a_attn", "a_gelu", "a_cls"))
    y = h.permute(0, 2, 3, 1).reshape(B, 1, -1)
    y = F.linear(y, rp(sd["patch_to_embedding.weight"]), sd["patch_to_embedding.bias"])
    x = torch.cat((sd["cls_token"].expand(B, -1, -1), y), 1) + _pos_rows(sd, pos_index, B)
    dim, heads = 1024, 8
    n = 2
    for l in range(6):
        p = f"transformer.layers.{l}."
        hh = F.layer_norm(x, (dim,), sd[p + "0.fn.norm.weight"], sd[p + "0.fn.norm.bias"], LN_EPS)
        qkv = F.linear(ln(hh), rw(sd[p + "0.fn.fn.to_qkv.weight"]))
        q, k, v = qkv.view(B, n, 3, heads, dim // heads).permute(2, 0, 3, 1, 4)
        att = (torch.einsum("bhid,bhjd->bhij", q, k) * dim ** -0.5).softmax(dim=-1)
        o = torch.einsum("bhij,bhjd->bhid", att, v).permute(0, 2, 1, 3).reshape(B, n, dim)
        x = F.linear(at(o), rw(sd[p + "0.fn.fn.to_out.weight"]), sd[p + "0.fn.fn.to_out.bias"]) + x
        hh = F.layer_norm(x, (dim,), sd[p + "1.fn.norm.weight"], sd[p + "1.fn.norm.bias"], LN_EPS)
        hh = F.gelu(F.linear(ln(hh), rw(sd[p + "1.fn.fn.net.0.weight"]), sd[p + "1.fn.fn.net.0.bias"]))
        x = F.linear(ge(hh), rw(sd[p + "1.fn.fn.net.2.weight"]), sd[p + "1.fn.fn.net.2.bias"]) + x
    c = cl(x[:, 0])
    hh = F.relu(F.linear(c, rw(sd["mlp_head.0.weight"]), sd["mlp_head.0.bias"]))
    return F.linear(hh, sd["mlp_head.2.weight"], sd["mlp_head.2.bias"])


def dp(a, b):
    return float((torch.sigmoid(a) - torch.sigmoid(b)).abs().max())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=64, help="crops of golden_b256's seed-3 batch")
    ap.add_argument("--threads", type=int, default=8)
    args = ap.parse_args()
    torch.set_num_threads(args.threads)
    sd = make_state_dict(0)
    crops = make_crops(256, seed=3)[: args.n]
    img = normalize_u8(crops)
    pos = np.arange(args.n) % 32
    ref = forward_fp32(sd, img, pos)
    allb = {k: "bf16" for k in POINTS}
    allh = {k: "fp16" for k in POINTS}
    print(f"all bf16: {dp(forward_policy(sd, img, pos, allb), ref):.3e}")
    print(f"all fp16: {dp(forward_policy(sd, img, pos, allh), ref):.3e}")
    groups = {
        "input": ["input"],
        "conv weights": [f"w_conv{i}" for i in range(17)],
        "conv acts 0-2 (224)": [f"a_conv{i}" for i in range(3)],
        "conv acts 3-5 (112)": [f"a_conv{i}" for i in range(3, 6)],
        "conv acts 6-8 (56)": [f"a_conv{i}" for i in range(6, 9)],
        "conv acts 9-12 (28)": [f"a_conv{i}" for i in range(9, 13)],
        "conv acts 13-16 (14)": [f"a_conv{i}" for i in range(13, 17)],
        "w_patch": ["w_patch"], "w_tail": ["w_tail"], "a_ln": ["a_ln"], "a_attn": ["a_attn"],
        "a_gelu": ["a_gelu"], "a_cls": ["a_cls"],
    }
    print(f"{'group':24s} {'only this bf16':>15s} {'all bf16 but this fp32':>24s} {'all bf16 but this fp16':>24s}")
    for g, pts in groups.items():
        only = dp(forward_policy(sd, img, pos, {k: "bf16" for k in pts}), ref)
        but32 = dp(forward_policy(sd, img, pos, {**allb, **{k: "fp32" for k in pts}}), ref)
        but16 = dp(forward_policy(sd, img, pos, {**allb, **{k: "fp16" for k in pts}}), ref)
        print(f"{g:24s} {only:15.3e} {but32:24.3e} {but16:24.3e}", flush=True)
    # candidate mixed policies
    tail = ["w_patch", "w_tail", "a_ln", "a_attn", "a_gelu", "a_cls"]
    cands = {
        "conv stack bf16, tail fp16": {**allb, **{k: "fp16" for k in tail}},
        "conv stack bf16 + a_conv16 fp16, tail fp16": {**allb, **{k: "fp16" for k in tail + ['a_conv16']}},
        "conv weights fp16, rest bf16": {**allb, **{f"w_conv{i}": "fp16" for i in range(17)}},
    }
    for name, pol in cands.items():
        print(f"{name:44s} {dp(forward_policy(sd, img, pos, pol), ref):.3e}", flush=True)


if __name__ == "__main__":
    main()
