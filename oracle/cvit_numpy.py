"""ORACLE (test infrastructure only): an independent numpy fp32 restatement of
the reference CViT forward (CViT-main/model/cvit.py:167-179), NHWC layout,
conv as an explicit im2col matmul.  It shares no code with the torch
restatement, so agreement of the two (and of both with the reference's
goldens) pins the oracle.  Sized for a handful of crops (~1-2 s per crop).
"""
from __future__ import annotations

import math

import numpy as np

from .cvit_torch import BN_EPS, LN_EPS, MEAN, POOL_AFTER, STD, stem_indices

f32 = np.float32


def normalize_u8(crops_u8: np.ndarray) -> np.ndarray:
    """uint8 NHWC -> normalised fp32 NHWC (cvit_prediction.py:209-215)."""
    x = crops_u8.astype(f32) / f32(255.0)
    return ((x - np.asarray(MEAN, f32)) / np.asarray(STD, f32)).astype(f32)


def conv3x3(x: np.ndarray, w: np.ndarray, b: np.ndarray) -> np.ndarray:
    """x [B,H,W,Ci], w [Co,Ci,3,3] (PyTorch layout), padding 1 -> [B,H,W,Co]."""
    B, H, W, Ci = x.shape
    xp = np.zeros((B, H + 2, W + 2, Ci), f32)
    xp[:, 1:-1, 1:-1] = x
    cols = np.empty((B, H, W, 9, Ci), f32)
    for ky in range(3):
        for kx in range(3):
            cols[:, :, :, ky * 3 + kx] = xp[:, ky:ky + H, kx:kx + W]
    wm = w.transpose(2, 3, 1, 0).reshape(9 * Ci, -1).astype(f32)   # [(ky,kx,ci), co]
    return (cols.reshape(-1, 9 * Ci) @ wm).reshape(B, H, W, -1) + b.astype(f32)


def maxpool2(x: np.ndarray) -> np.ndarray:
    B, H, W, C = x.shape
    return x.reshape(B, H // 2, 2, W // 2, 2, C).max(axis=(2, 4))


def layer_norm(x, g, b):
    mu = x.mean(-1, keepdims=True, dtype=np.float64).astype(f32)
    var = ((x - mu) ** 2).mean(-1, keepdims=True, dtype=np.float64).astype(f32)
    return ((x - mu) / np.sqrt(var + f32(LN_EPS)) * g + b).astype(f32)


def gelu(x):
    erf = np.vectorize(math.erf, otypes=[np.float64])
    return (0.5 * x * (1.0 + erf(x.astype(np.float64) / math.sqrt(2.0)))).astype(f32)


def softmax(x, axis=-1):
    e = np.exp(x - x.max(axis=axis, keepdims=True))
    return (e / e.sum(axis=axis, keepdims=True)).astype(f32)


def forward(sd, x_nhwc: np.ndarray, pos_index=None) -> np.ndarray:
    """Normalised fp32 NHWC [B,224,224,3] -> logits [B,2]."""
    sd = {k: np.asarray(v) for k, v in sd.items()}
    h = x_nhwc.astype(f32)
    for i, (ci, bi) in enumerate(stem_indices()):
        p, q = f"features.{ci}.", f"features.{bi}."
        h = conv3x3(h, sd[p + "weight"], sd[p + "bias"])
        h = (h - sd[q + "running_mean"]) / np.sqrt(sd[q + "running_var"] + f32(BN_EPS)) * sd[q + "weight"] \
            + sd[q + "bias"]
        h = np.maximum(h.astype(f32), 0)
        if i in POOL_AFTER:
            h = maxpool2(h)
    B = h.shape[0]
    y = h.reshape(B, -1) @ sd["patch_to_embedding.weight"].T + sd["patch_to_embedding.bias"]   # NHWC flatten
    pidx = np.arange(B) if pos_index is None else np.asarray(pos_index)
    pos = sd["pos_embedding"][pidx, 0]                                                          # [B,dim]
    x = np.stack([sd["cls_token"][0, 0][None].repeat(B, 0), y], 1) + pos[:, None, :]
    dim, heads = x.shape[-1], 8
    dh = dim // heads
    for l in range(6):
        p = f"transformer.layers.{l}."
        t = layer_norm(x, sd[p + "0.fn.norm.weight"], sd[p + "0.fn.norm.bias"])
        qkv = t @ sd[p + "0.fn.fn.to_qkv.weight"].T                                             # [B,2,3*dim]
        q, k, v = (qkv[..., j * dim:(j + 1) * dim].reshape(B, 2, heads, dh).transpose(0, 2, 1, 3) for j in range(3))
        a = softmax(q @ k.transpose(0, 1, 3, 2) * f32(dim ** -0.5))
        o = (a @ v).transpose(0, 2, 1, 3).reshape(B, 2, dim)
        x = x + o @ sd[p + "0.fn.fn.to_out.weight"].T + sd[p + "0.fn.fn.to_out.bias"]
        t = layer_norm(x, sd[p + "1.fn.norm.weight"], sd[p + "1.fn.norm.bias"])
        t = gelu(t @ sd[p + "1.fn.fn.net.0.weight"].T + sd[p + "1.fn.fn.net.0.bias"])
        x = (x + t @ sd[p + "1.fn.fn.net.2.weight"].T + sd[p + "1.fn.fn.net.2.bias"]).astype(f32)
    c = x[:, 0]
    hh = np.maximum(c @ sd["mlp_head.0.weight"].T + sd["mlp_head.0.bias"], 0)
    return (hh @ sd["mlp_head.2.weight"].T + sd["mlp_head.2.bias"]).astype(f32)
