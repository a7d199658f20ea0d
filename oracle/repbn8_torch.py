"""ORACLE (test infrastructure, never shipped or measured as the product).

CPU restatement of the CViT RepBn8 variant,
``CViT-main/model/cvit_GGCA_ADD_DEConv_RepBn8.py::CViT`` (:343-455), written
functionally over its state_dict with the PyTorch CPU ops the reference calls:

* ``deconv_fold``  - DEConv's eval weight algebra (:320-340 with Conv2d_cd
                      :214-229, Conv2d_hd :287-299, Conv2d_vd :302-316,
                      Conv2d_ad :232-247): five kernels -> one 3x3 + bias.
* ``ggca``         - GGCA(512, 7, 7) (:144-207).
* ``forward_fp32`` - CViT.forward (:432-455), fp32.  The FeedForward PreNorm
                      is LinearNorm, whose eval path is LayerNorm(eps 1e-6)
                      (:22-46, :48-59); the attention PreNorm is
                      nn.LayerNorm (eps 1e-5, :61-69).
* ``forward_emulated`` - the same with operands rounded to 16 bits where the
                      gfx950 path rounds them.

Pinned against tests/golden/repbn8_golden.npz, produced from the
reference's own class code (tools/make_golden_repbn8.py; the module is
CUDA-only, so that script runs its classes on the CPU with the CUDA scratch
factory replaced — see its header).
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from .cvit_torch import BN_EPS, _pos_rows, _transformer, round_to, to_torch_sd

LAYERS = [  # fac_fake_amd.weights.REPBN8_LAYERS, restated: (seq, idx, kind, cin, cout, bn, relu, pool)
    ("features1", 0, "conv", 3, 32, 1, True, False), ("features1", 3, "deconv", 32, 32, 4, True, False),
    ("features1", 6, "deconv", 32, 32, 7, True, True), ("features1", 10, "conv", 32, 64, 11, True, False),
    ("features1", 13, "deconv", 64, 64, 14, True, False), ("features1", 16, "deconv", 64, 64, 17, True, True),
    ("features1", 20, "conv", 64, 128, 21, True, False), ("features1", 23, "deconv", 128, 128, 24, True, False),
    ("features1", 26, "conv", 128, 128, None, False, False), ("features1", 27, "deconv", 128, 128, None, True, True),
    ("features1", 30, "conv", 128, 256, 31, True, False), ("features1", 33, "deconv", 256, 256, 34, True, False),
    ("features1", 36, "deconv", 256, 256, 37, True, False), ("features1", 39, "deconv", 256, 256, 40, True, True),
    ("features2", 0, "conv", 256, 512, 1, True, False), ("features2", 3, "deconv", 512, 512, 4, True, False),
    ("features2", 6, "deconv", 512, 512, 7, True, False), ("features2", 9, "deconv", 512, 512, 10, True, True)]
FF_LN_EPS = 1e-6  # LinearNorm.norm1 = partial(nn.LayerNorm, eps=1e-6) (:48)


def deconv_fold(sd, p):
    """DEConv.forward's weight and bias (:329-338), in the reference's op order."""
    w1 = sd[p + ".conv1_1.conv.weight"]
    o, i = w1.shape[:2]
    t = w1.reshape(o, i, 9)
    cd = torch.zeros(o, i, 9)
    cd[:, :, :] = t[:, :, :]
    cd[:, :, 4] = t[:, :, 4] - t[:, :, :].sum(2)                       # Conv2d_cd (:221-228)
    h = sd[p + ".conv1_2.conv.weight"]
    hd = torch.zeros(o, i, 9)
    hd[:, :, [0, 3, 6]] = h[:, :, :]
    hd[:, :, [2, 5, 8]] = -h[:, :, :]                                  # Conv2d_hd (:292-297)
    v = sd[p + ".conv1_3.conv.weight"]
    vd = torch.zeros(o, i, 9)
    vd[:, :, [0, 1, 2]] = v[:, :, :]
    vd[:, :, [6, 7, 8]] = -v[:, :, :]                                  # Conv2d_vd (:310-315)
    a = sd[p + ".conv1_4.conv.weight"].reshape(o, i, 9)
    ad = a - 1.0 * a[:, :, [3, 0, 1, 6, 4, 2, 7, 8, 5]]                # Conv2d_ad, theta 1 (:242-246)
    w = (cd.reshape(o, i, 3, 3) + hd.reshape(o, i, 3, 3) + vd.reshape(o, i, 3, 3) + ad.reshape(o, i, 3, 3)
         + sd[p + ".conv1_5.weight"])
    b = (sd[p + ".conv1_1.conv.bias"] + sd[p + ".conv1_2.conv.bias"] + sd[p + ".conv1_3.conv.bias"]
         + sd[p + ".conv1_4.conv.bias"] + sd[p + ".conv1_5.bias"])
    return w, b


def layer_weights(sd, layer):
    seq, idx, kind, *_ = layer
    p = f"{seq}.{idx}"
    if kind == "conv":
        return sd[p + ".weight"], sd[p + ".bias"]
    return deconv_fold(sd, p)


def _shared_conv(sd, v):
    """GGCA.shared_conv (:160-167) on [N, 128, h, w]."""
    q = "ggca.shared_conv."
    v = F.conv2d(v, sd[q + "0.weight"], sd[q + "0.bias"])
    v = F.batch_norm(v, sd[q + "1.running_mean"], sd[q + "1.running_var"], sd[q + "1.weight"], sd[q + "1.bias"],
                     False, 0.1, BN_EPS)
    return F.conv2d(F.relu(v), sd[q + "3.weight"], sd[q + "3.bias"])


def ggca(sd, x, groups=4):
    """GGCA.forward (:172-207) on fp32 NCHW [B, 512, 7, 7]; returns x * att_h * att_w."""
    B, C, H, W = x.shape
    gc = C // groups
    xg = x.reshape(B * groups, gc, H, W)
    h_avg = F.adaptive_avg_pool2d(xg, (H, 1))
    h_max = F.adaptive_max_pool2d(xg, (H, 1))
    w_avg = F.adaptive_avg_pool2d(xg, (1, W))
    w_max = F.adaptive_max_pool2d(xg, (1, W))
    att_h = torch.sigmoid(_shared_conv(sd, h_avg) + _shared_conv(sd, h_max)).view(B, groups, gc, H, 1)
    att_w = torch.sigmoid(_shared_conv(sd, w_avg) + _shared_conv(sd, w_max)).view(B, groups, gc, 1, W)
    out = x.view(B, groups, gc, H, W) * att_h * att_w
    return out.view(B, C, H, W)


def _tail(sd, h, pos_index, lin=None, act_round=None):
    B = h.shape[0]
    y = h.permute(0, 2, 3, 1).reshape(B, 1, -1)          # 'b c (h p1) (w p2) -> b (h w) (p1 p2 c)'
    lin = lin or (lambda inp, w, b=None: F.linear(inp, w, b))
    y = lin(y, sd["patch_to_embedding.weight"], sd["patch_to_embedding.bias"])
    x = torch.cat((sd["cls_token"].expand(B, -1, -1), y), 1) + _pos_rows(sd, pos_index, B)
    x = _transformer(sd, x, lin=lin, act_round=act_round, ff_norm="1.fn.norm.norm1", ff_eps=FF_LN_EPS)
    c = x[:, 0]
    if act_round is not None:
        c = act_round(c)
    hid = F.relu(lin(c, sd["mlp_head.0.weight"], sd["mlp_head.0.bias"]))
    return F.linear(hid, sd["mlp_head.2.weight"], sd["mlp_head.2.bias"])


@torch.no_grad()
def forward_fp32(sd, img: torch.Tensor, pos_index=None, return_features: bool = False):
    """The reference CViT.forward (:432-455) on normalised fp32 NCHW input."""
    sd = to_torch_sd(sd)
    h = img.float()
    for layer in LAYERS:
        seq, idx, kind, ci, co, bn, relu, pool = layer
        w, b = layer_weights(sd, layer)
        h = F.conv2d(h, w, b, padding=1)
        if bn is not None:
            q = f"{seq}.{bn}."
            h = F.batch_norm(h, sd[q + "running_mean"], sd[q + "running_var"], sd[q + "weight"], sd[q + "bias"],
                             False, 0.1, BN_EPS)
        if relu:
            h = F.relu(h)
        if pool:
            h = F.max_pool2d(h, 2, 2)
    f2 = h
    weighted = h * ggca(sd, h)                            # x1 = ggca(x); x = x * x1 (:436-437)
    out = _tail(sd, weighted, pos_index)
    return (out, f2, weighted) if return_features else out


def fold_layer(sd, layer):
    """Conv (+ DEConv fold) + eval BN folded in fp32: W' = W s, b' = (b - mean) s + beta."""
    seq, idx, kind, ci, co, bn, relu, pool = layer
    w, b = layer_weights(sd, layer)
    if bn is None:
        return w, b
    q = f"{seq}.{bn}."
    s = sd[q + "weight"] / torch.sqrt(sd[q + "running_var"] + torch.tensor(BN_EPS, dtype=torch.float32))
    return w * s.view(-1, 1, 1, 1), (b - sd[q + "running_mean"]) * s + sd[q + "bias"]


@torch.no_grad()
def forward_emulated(sd, img: torch.Tensor, pos_index=None, dtype: str = "bf16", return_features: bool = False):
    """The gfx950 path's rounding points: 16-bit normalised input, folded conv
    weights and every conv output; the GGCA-weighted features; the tail's
    weight matrices and GEMM inputs (fp32 accumulation, statistics,
    residual stream and epilogues)."""
    sd = to_torch_sd(sd)
    r = lambda t: round_to(t, dtype)  # noqa: E731
    h = r(img.float())
    for layer in LAYERS:
        w, b = fold_layer(sd, layer)
        h = F.conv2d(h, r(w), b, padding=1)
        if layer[6]:
            h = F.relu(h)
        if layer[7]:
            h = F.max_pool2d(h, 2, 2)
        h = r(h)
    f2 = h
    weighted = r(h * ggca(sd, h))
    lin = lambda inp, w, b=None: F.linear(r(inp), r(w), b)  # noqa: E731
    out = _tail(sd, weighted, pos_index, lin=lin)
    return (out, f2, weighted) if return_features else out
