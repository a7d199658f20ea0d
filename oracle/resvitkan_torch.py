"""ORACLE (test infrastructure, never shipped or measured as the product).

CPU restatement of the ResVitKan forward (BASELINE config 5,
``CViT-main/ResVitKan/ResVitKan.py:284-329`` with ``kan.py``), functional
over a state_dict with the PyTorch CPU ops the reference modules call:

* ``resnet50_fp32``  - ``ResNet.forward`` (ResVitKan.py:232-247): 7x7/2 conv,
                       BN, ReLU, 3x3/2 max-pool, Bottleneck x [3,4,6,3]
                       (:124-152 — note the ReLU after bn3 *before* the
                       residual add, then ReLU again), ``channel`` 1x1 + bn2.
* ``kan_linear_fp32``- ``KANLinear.forward`` (kan.py:189-206) with
                       ``b_splines`` (kan.py:90-132) in the reference's op order.
* ``forward_fp32``   - ``CViT.forward`` (ResVitKan.py:316-329).  Pinned
                       against outputs of the reference module itself
                       (tests/golden/resvitkan_*, tools/make_golden_resvitkan.py).
* ``forward_emulated``- the gfx950 path's rounding points (16-bit folded
                       weights and conv outputs, the residual added in fp32
                       to the 16-bit block input, fp32 KAN).

Only tests/, __graft_entry__.smoke() and bench.py may import this package.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from .cvit_torch import LN_EPS, _pos_rows, _transformer, round_to, to_torch_sd

BN_EPS = 1e-5                                   # nn.BatchNorm2d default (ResVitKan.py:129-135, :193-203)
LAYERS = [(64, 3, 1), (128, 4, 2), (256, 6, 2), (512, 3, 2)]  # resnet50 (ResVitKan.py:259-264)


def blocks():
    """(prefix, stride, has_downsample) per Bottleneck (ResVitKan.py:216-230)."""
    out, inplanes = [], 64
    for li, (planes, n, stride) in enumerate(LAYERS):
        for b in range(n):
            s = stride if b == 0 else 1
            out.append((f"features.layer{li + 1}.{b}", s, b == 0 and (s != 1 or inplanes != planes * 4)))
            inplanes = planes * 4
    return out


def _bn(sd, p, h):
    return F.batch_norm(h, sd[p + ".running_mean"], sd[p + ".running_var"], sd[p + ".weight"], sd[p + ".bias"],
                        False, 0.1, BN_EPS)


@torch.no_grad()
def resnet50_fp32(sd, img: torch.Tensor, taps: list | None = None) -> torch.Tensor:
    """With `taps`: the max-pool output, every Bottleneck's output and the
    bn2 output are appended (what forward hooks on the reference's maxpool,
    layerN[b] and bn2 see)."""
    sd = to_torch_sd(sd)
    tap = taps.append if taps is not None else (lambda t: None)
    x = F.relu(_bn(sd, "features.bn1", F.conv2d(img.float(), sd["features.conv1.weight"], stride=2, padding=3)))
    x = F.max_pool2d(x, 3, 2, 1)
    tap(x)
    for p, s, ds in blocks():
        res = x
        out = F.relu(_bn(sd, p + ".bn1", F.conv2d(x, sd[p + ".conv1.weight"])))
        out = F.relu(_bn(sd, p + ".bn2", F.conv2d(out, sd[p + ".conv2.weight"], stride=s, padding=1)))
        out = F.relu(_bn(sd, p + ".bn3", F.conv2d(out, sd[p + ".conv3.weight"])))
        if ds:
            res = _bn(sd, p + ".downsample.1", F.conv2d(x, sd[p + ".downsample.0.weight"], stride=s))
        x = F.relu(out + res)
        tap(x)
    y = _bn(sd, "features.bn2", F.conv2d(x, sd["features.channel.weight"]))
    tap(y)
    return y


def b_splines(x: torch.Tensor, grid: torch.Tensor, order: int = 3) -> torch.Tensor:
    """kan.py:90-132: x [B, in], grid [in, n_knots] -> bases [B, in, n_knots - 1 - order]."""
    x = x.unsqueeze(-1)
    bases = ((x >= grid[:, :-1]) & (x < grid[:, 1:])).to(x.dtype)
    for k in range(1, order + 1):
        bases = ((x - grid[:, :-(k + 1)]) / (grid[:, k:-1] - grid[:, :-(k + 1)]) * bases[:, :, :-1]) + (
            (grid[:, k + 1:] - x) / (grid[:, k + 1:] - grid[:, 1:(-k)]) * bases[:, :, 1:])
    return bases.contiguous()


@torch.no_grad()
def kan_linear_fp32(sd, prefix: str, x: torch.Tensor) -> torch.Tensor:
    """KANLinear.forward (kan.py:189-206)."""
    bw, sw = sd[prefix + ".base_weight"], sd[prefix + ".spline_weight"]
    scaled = sw * sd[prefix + ".spline_scaler"].unsqueeze(-1)
    base = F.linear(F.silu(x), bw)
    spline = F.linear(b_splines(x, sd[prefix + ".grid"]).view(x.size(0), -1), scaled.view(bw.shape[0], -1))
    return base + spline


def _kan_head_tail(sd, hidden):
    h = kan_linear_fp32(sd, "kan_head.3.layers.0", hidden)
    return kan_linear_fp32(sd, "kan_head.3.layers.1", h)


@torch.no_grad()
def forward_fp32(sd, img: torch.Tensor, pos_index=None) -> torch.Tensor:
    """ResVitKan CViT.forward (ResVitKan.py:316-329), eval mode (Dropout = identity)."""
    sd = to_torch_sd(sd)
    f = resnet50_fp32(sd, img)
    B = f.shape[0]
    y = f.permute(0, 2, 3, 1).reshape(B, 1, -1)   # rearrange 'b c (h p1) (w p2) -> b (h w) (p1 p2 c)'
    y = F.linear(y, sd["patch_to_embedding.weight"], sd["patch_to_embedding.bias"])
    x = torch.cat((sd["cls_token"].expand(B, -1, -1), y), 1) + _pos_rows(sd, pos_index, B)
    x = _transformer(sd, x)
    hid = F.relu(F.linear(x[:, 0], sd["kan_head.0.weight"], sd["kan_head.0.bias"]))
    return _kan_head_tail(sd, hid)


def fold_bn(sd, conv_key: str, bn_prefix: str):
    s = sd[bn_prefix + ".weight"] / torch.sqrt(sd[bn_prefix + ".running_var"] + torch.tensor(BN_EPS))
    w = sd[conv_key] * s.view(-1, 1, 1, 1)
    b = (torch.zeros_like(s) - sd[bn_prefix + ".running_mean"]) * s + sd[bn_prefix + ".bias"]
    return w, b


@torch.no_grad()
def resnet50_emulated(sd, img: torch.Tensor, dtype: str = "bf16", taps: list | None = None) -> torch.Tensor:
    """ResNet-50 stem at the HIP path's rounding points (fac_conv_nd epilogues);
    `taps` as in resnet50_fp32."""
    sd = to_torch_sd(sd)
    tap = taps.append if taps is not None else (lambda t: None)
    r = lambda t: round_to(t, dtype)  # noqa: E731

    def conv(x, ck, bnp, stride=1, pad=0, relu=True, res=None):
        w, b = fold_bn(sd, ck, bnp)
        v = F.conv2d(x, r(w), b, stride=stride, padding=pad)
        if relu:
            v = F.relu(v)
        if res is not None:
            v = F.relu(v + res)
        return r(v)

    x = conv(r(img.float()), "features.conv1.weight", "features.bn1", 2, 3)
    x = F.max_pool2d(x, 3, 2, 1)
    tap(x)
    for p, s, ds in blocks():
        res = conv(x, p + ".downsample.0.weight", p + ".downsample.1", s, 0, relu=False) if ds else x
        out = conv(x, p + ".conv1.weight", p + ".bn1")
        out = conv(out, p + ".conv2.weight", p + ".bn2", s, 1)
        x = conv(out, p + ".conv3.weight", p + ".bn3", res=res)
        tap(x)
    y = conv(x, "features.channel.weight", "features.bn2", relu=False)
    tap(y)
    return y


@torch.no_grad()
def forward_emulated(sd, img: torch.Tensor, pos_index=None, dtype: str = "bf16", return_hidden: bool = False):
    sd = to_torch_sd(sd)
    r = lambda t: round_to(t, dtype)  # noqa: E731
    f = resnet50_emulated(sd, img, dtype)
    B = f.shape[0]
    y = f.permute(0, 2, 3, 1).reshape(B, 1, -1)
    y = F.linear(y, r(sd["patch_to_embedding.weight"]), sd["patch_to_embedding.bias"])
    x = torch.cat((sd["cls_token"].expand(B, -1, -1), y), 1) + _pos_rows(sd, pos_index, B)
    lin = lambda inp, w, b=None: F.linear(inp, r(w), b)  # noqa: E731
    x = _transformer(sd, x, lin=lin, act_round=r)
    hid = F.relu(F.linear(r(x[:, 0]), r(sd["kan_head.0.weight"]), sd["kan_head.0.bias"]))
    out = _kan_head_tail(sd, hid)
    return (out, hid) if return_hidden else out


__all__ = ["resnet50_fp32", "kan_linear_fp32", "b_splines", "forward_fp32", "resnet50_emulated", "forward_emulated",
           "blocks", "LN_EPS"]
