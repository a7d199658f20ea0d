"""ORACLE (test infrastructure, never shipped or measured as the product).

CPU restatement of the reference CViT forward, ``CViT-main/model/cvit.py``,
written functionally over a state_dict with the same PyTorch CPU ops the
reference module calls, so it executes the same kernels:

* ``forward_fp32``   - the reference arithmetic (cvit.py:167-179), fp32.
                        Pinned against goldens produced by the reference
                        itself (tests/golden/, tools/make_golden.py).  Also
                        the ``cpu_baseline`` leg of bench.py (kind "port").
* ``forward_emulated``- the same network with operands rounded to bf16/fp16
                        exactly where the gfx950 path rounds them (BN folded
                        then rounded weights, 16-bit activations between
                        layers, fp32 accumulation and epilogues).  Used to
                        check the HIP kernels tightly; the fp32 goldens check
                        end-to-end parity.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline may import
this package.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

MEAN = (0.485, 0.456, 0.406)     # cvit_prediction.py:41
STD = (0.229, 0.224, 0.225)      # cvit_prediction.py:42
BN_EPS = 1e-5                    # nn.BatchNorm2d default (cvit.py:89..146)
LN_EPS = 1e-5                    # nn.LayerNorm default (cvit.py:16)
STEM = [(3, 32), (32, 32), (32, 32), (32, 64), (64, 64), (64, 64), (64, 128), (128, 128), (128, 128),
        (128, 256), (256, 256), (256, 256), (256, 256), (256, 512), (512, 512), (512, 512), (512, 512)]
POOL_AFTER = {2, 5, 8, 12, 16}   # MaxPool2d(2,2) at cvit.py:97,108,119,133,147


def stem_indices():
    """(conv, bn) nn.Sequential indices of the 17 convs (cvit.py:86-148)."""
    out, idx = [], 0
    for i in range(17):
        out.append((idx, idx + 1))
        idx += 3 + (1 if i in POOL_AFTER else 0)
    return out


def to_torch_sd(sd) -> dict:
    return {k: torch.as_tensor(v) for k, v in sd.items()}


def normalize_u8(crops_u8) -> torch.Tensor:
    """uint8 NHWC -> normalised fp32 NCHW, in the reference's op order
    (cvit_prediction.py:209-215: .float(), permute, /255., Normalize)."""
    x = torch.as_tensor(crops_u8).float().permute(0, 3, 1, 2)
    x = x / 255.
    mean = torch.tensor(MEAN, dtype=torch.float32).view(1, 3, 1, 1)
    std = torch.tensor(STD, dtype=torch.float32).view(1, 3, 1, 1)
    return ((x - mean) / std).contiguous()


def _pos_rows(sd, pos_index, B):
    pos = sd["pos_embedding"]  # [32,1,dim]
    if pos_index is None:
        return pos[0:B]        # cvit.py:175 (raises past 32 crops, like the reference)
    return pos[torch.as_tensor(pos_index, dtype=torch.long)]


def _transformer(sd, x, depth=6, heads=8, lin=None, act_round=None, ff_norm="1.fn.norm", ff_eps=LN_EPS):
    """6 x {x += to_out(attn(LN(x))); x += FF(LN(x))} (cvit.py:5-78).  ff_norm /
    ff_eps: the FeedForward PreNorm's LayerNorm (the RepBn8 variant's
    LinearNorm evaluates LayerNorm(eps 1e-6) at ``1.fn.norm.norm1``)."""
    lin = lin or (lambda inp, w, b=None: F.linear(inp, w, b))
    rnd = act_round or (lambda t: t)
    B, n, dim = x.shape
    scale = dim ** -0.5        # cvit.py:38 uses dim, not the head width
    for l in range(depth):
        p = f"transformer.layers.{l}."
        h = F.layer_norm(x, (dim,), sd[p + "0.fn.norm.weight"], sd[p + "0.fn.norm.bias"], LN_EPS)
        qkv = lin(rnd(h), sd[p + "0.fn.fn.to_qkv.weight"])
        q, k, v = qkv.view(B, n, 3, heads, dim // heads).permute(2, 0, 3, 1, 4)
        att = (torch.einsum("bhid,bhjd->bhij", q, k) * scale).softmax(dim=-1)
        o = torch.einsum("bhij,bhjd->bhid", att, v).permute(0, 2, 1, 3).reshape(B, n, dim)
        x = lin(rnd(o), sd[p + "0.fn.fn.to_out.weight"], sd[p + "0.fn.fn.to_out.bias"]) + x
        h = F.layer_norm(x, (dim,), sd[p + ff_norm + ".weight"], sd[p + ff_norm + ".bias"], ff_eps)
        h = F.gelu(lin(rnd(h), sd[p + "1.fn.fn.net.0.weight"], sd[p + "1.fn.fn.net.0.bias"]))
        x = lin(rnd(h), sd[p + "1.fn.fn.net.2.weight"], sd[p + "1.fn.fn.net.2.bias"]) + x
    return x


@torch.no_grad()
def forward_fp32(sd, img: torch.Tensor, pos_index=None, return_features: bool = False):
    """Reference CViT.forward (cvit.py:167-179) on normalised fp32 NCHW input."""
    sd = to_torch_sd(sd)
    h = img.float()
    feats = []
    for i, (ci, bi) in enumerate(stem_indices()):
        p, q = f"features.{ci}.", f"features.{bi}."
        h = F.conv2d(h, sd[p + "weight"], sd[p + "bias"], padding=1)
        h = F.batch_norm(h, sd[q + "running_mean"], sd[q + "running_var"], sd[q + "weight"], sd[q + "bias"],
                         False, 0.1, BN_EPS)
        h = F.relu(h)
        if i in POOL_AFTER:
            h = F.max_pool2d(h, 2, 2)
        feats.append(h)
    out = tail_fp32(sd, h, pos_index)
    return (out, feats) if return_features else out


@torch.no_grad()
def tail_fp32(sd, h: torch.Tensor, pos_index=None):
    """Stem output [B,512,7,7] -> logits: cvit.py:170-179 in fp32."""
    sd = to_torch_sd(sd)
    B = h.shape[0]
    y = h.permute(0, 2, 3, 1).reshape(B, 1, -1)  # 'b c (h p1) (w p2) -> b (h w) (p1 p2 c)' with h=w=1
    y = F.linear(y, sd["patch_to_embedding.weight"], sd["patch_to_embedding.bias"])
    x = torch.cat((sd["cls_token"].expand(B, -1, -1), y), 1)
    x = x + _pos_rows(sd, pos_index, B)
    x = _transformer(sd, x)
    c = x[:, 0]
    return F.linear(F.relu(F.linear(c, sd["mlp_head.0.weight"], sd["mlp_head.0.bias"])), sd["mlp_head.2.weight"],
                    sd["mlp_head.2.bias"])


def round_to(t: torch.Tensor, dtype: str) -> torch.Tensor:
    td = {"bf16": torch.bfloat16, "fp16": torch.float16}[dtype]
    return t.to(td).float()


def fold_bn(sd, ci, bi):
    """BN folded into conv (fp32, same formula and op order as cvit_abi.hip)."""
    p, q = f"features.{ci}.", f"features.{bi}."
    s = sd[q + "weight"] / torch.sqrt(sd[q + "running_var"] + torch.tensor(BN_EPS, dtype=torch.float32))
    w = sd[p + "weight"] * s.view(-1, 1, 1, 1)
    b = (sd[p + "bias"] - sd[q + "running_mean"]) * s + sd[q + "bias"]
    return w, b


def conv3x3_wino_f23(h: torch.Tensor, w: torch.Tensor, b: torch.Tensor, dtype: str) -> torch.Tensor:
    """Conv2d(3x3, pad 1) + bias of a 16-bit-valued NCHW input as the HIP
    path's Winograd F(2,3) along x computes it (fac_fake_amd/csrc/wino.hip):
    per output pair (2p, 2p+1) and input row, d_x = x-columns 2p-1 .. 2p+2
    (zero padded), V = (d0-d2, d1+d2, d2-d1, d1-d3) in fp32 rounded to 16
    bits; U = (g0, (g0+g1+g2)/2, (g0-g1+g2)/2, g2) of each folded kernel row
    in fp64 rounded to 16 bits; M_j = sum over (channel, kernel row) of
    U_j V_j in fp32; out = (M0+M1+M2, M1-M2-M3) + bias, fp32 (before ReLU)."""
    N, C, H, W = h.shape
    d = F.pad(h.float(), (1, 1, 1, 1)).unfold(3, 4, 2)          # [N, C, H+2, W/2, 4]
    d0, d1, d2, d3 = d.unbind(-1)
    V = round_to(torch.stack([d0 - d2, d1 + d2, d2 - d1, d1 - d3], -1), dtype)   # [N, C, H+2, W/2, 4]
    g = w.double()
    g0, g1, g2 = g[..., 0], g[..., 1], g[..., 2]                 # [K, C, 3(ky)]
    U = round_to(torch.stack([g0, (g0 + g1 + g2) * 0.5, (g0 - g1 + g2) * 0.5, g2], -1).float(), dtype)
    M = sum(torch.einsum("kcj,ncypj->nkypj", U[:, :, ky], V[:, :, ky:ky + H]) for ky in range(3))
    m0, m1, m2, m3 = M.unbind(-1)                                # [N, K, H, W/2]
    out = torch.stack([m0 + m1 + m2, m1 - m2 - m3], -1).reshape(N, -1, H, W)
    return out + b.view(1, -1, 1, 1)


@torch.no_grad()
def forward_emulated(sd, img: torch.Tensor, pos_index=None, dtype: str = "bf16", return_features: bool = False,
                     wino=()):
    """The gfx950 path's arithmetic on the CPU: 16-bit operands, fp32 accumulate.

    Rounding points (cf. conv.hip / transformer.hip): the normalised input;
    every folded conv weight; every conv output after bias+ReLU(+pool); the
    patch-embed and transformer/head weight matrices; LayerNorm outputs; the
    attention output; the GELU output; the CLS rows entering the head.  fp32:
    conv/BN biases, the residual stream, QKV, softmax, LN statistics, the
    final 2048->2 layer and its input.
    """
    sd = to_torch_sd(sd)
    r = lambda t: round_to(t, dtype)  # noqa: E731
    h = r(img.float())
    feats = []
    for i, (ci, bi) in enumerate(stem_indices()):
        w, b = fold_bn(sd, ci, bi)
        if i in wino:   # conv layers (0-based) the HIP path runs as Winograd F(2,3)
            h = F.relu(conv3x3_wino_f23(h, w, b, dtype))
        else:
            h = F.relu(F.conv2d(h, r(w), b, padding=1))
        if i in POOL_AFTER:
            h = F.max_pool2d(h, 2, 2)
        h = r(h)
        feats.append(h)
    out = tail_emulated(sd, h, pos_index, dtype)
    return (out, feats) if return_features else out


@torch.no_grad()
def conv_block_emulated(sd, h: torch.Tensor, i: int, dtype: str = "bf16") -> torch.Tensor:
    """Conv i (0-based) alone on a 16-bit-valued NCHW input, HIP rounding points."""
    sd = to_torch_sd(sd)
    ci, bi = stem_indices()[i]
    w, b = fold_bn(sd, ci, bi)
    h = F.relu(F.conv2d(h, round_to(w, dtype), b, padding=1))
    if i in POOL_AFTER:
        h = F.max_pool2d(h, 2, 2)
    return round_to(h, dtype)


@torch.no_grad()
def tail_emulated(sd, h: torch.Tensor, pos_index=None, dtype: str = "bf16"):
    """Stem output (16-bit valued) -> logits with the HIP path's rounding points."""
    sd = to_torch_sd(sd)
    r = lambda t: round_to(t, dtype)  # noqa: E731
    B = h.shape[0]
    y = h.permute(0, 2, 3, 1).reshape(B, 1, -1)
    y = F.linear(y, r(sd["patch_to_embedding.weight"]), sd["patch_to_embedding.bias"])
    x = torch.cat((sd["cls_token"].expand(B, -1, -1), y), 1) + _pos_rows(sd, pos_index, B)
    lin = lambda inp, w, b=None: F.linear(inp, r(w), b)  # noqa: E731
    x = _transformer(sd, x, lin=lin, act_round=r)
    c = r(x[:, 0])
    hh = F.relu(F.linear(c, r(sd["mlp_head.0.weight"]), sd["mlp_head.0.bias"]))
    return F.linear(hh, sd["mlp_head.2.weight"], sd["mlp_head.2.bias"])
