"""Deterministic synthetic CViT weights and crops (counter-based splitmix64).

The reference ships no trained weights (``CViT-main/weight/`` is gitignored,
SURVEY.md §8c), so every parity test and the benchmark run on weights made
here.  The generator is pure integer arithmetic followed by exact float32
conversion, so this container, the GPU box and any C/C++ re-implementation
produce bit-identical tensors from ``(seed, tensor name)`` alone and no
weight file ever has to travel.

The state_dict layout (193 keys, same names, shapes and order) is the one
``CViT-main/model/cvit.py:80-165`` builds and ``cvit_train.py:210`` saves.
"""
from __future__ import annotations

import hashlib
from collections import OrderedDict

import numpy as np

_GOLDEN = np.uint64(0x9E3779B97F4A7C15)
_M1 = np.uint64(0xBF58476D1CE4E5B9)
_M2 = np.uint64(0x94D049BB133111EB)

# conv stem channel plan, cvit.py:86-148 (conv, BN, ReLU triples; pools after
# the 3rd, 6th, 9th, 13th and 17th conv)
STEM_CHANNELS = [(3, 32), (32, 32), (32, 32),
                 (32, 64), (64, 64), (64, 64),
                 (64, 128), (128, 128), (128, 128),
                 (128, 256), (256, 256), (256, 256), (256, 256),
                 (256, 512), (512, 512), (512, 512), (512, 512)]
POOL_AFTER = {2, 5, 8, 12, 16}          # 0-based conv index followed by MaxPool2d(2,2)


def stem_module_indices():
    """nn.Sequential indices of (conv, bn) for each of the 17 convs.

    Mirrors the Sequential at cvit.py:86-148: conv, BN, ReLU per conv plus a
    MaxPool after convs 3/6/9/13/17, giving conv indices 0,3,6 | 10,13,16 | ...
    """
    idx, out = 0, []
    for i in range(17):
        out.append((idx, idx + 1))
        idx += 3
        if i in POOL_AFTER:
            idx += 1
    return out


def splitmix64(counter: np.ndarray, seed: int) -> np.ndarray:
    """splitmix64 of ``seed + (counter+1)*golden`` (wrapping uint64)."""
    with np.errstate(over="ignore"):
        z = np.uint64(seed & 0xFFFFFFFFFFFFFFFF) + (counter.astype(np.uint64) + np.uint64(1)) * _GOLDEN
        z = (z ^ (z >> np.uint64(30))) * _M1
        z = (z ^ (z >> np.uint64(27))) * _M2
        return z ^ (z >> np.uint64(31))


def _stream_seed(seed: int, name: str) -> int:
    h = hashlib.sha256(f"{seed}:{name}".encode()).digest()
    return int.from_bytes(h[:8], "little")


def uniform(name: str, n: int, seed: int) -> np.ndarray:
    """n float32 values in [-1, 1) for stream ``name`` (exact: 24-bit grid)."""
    z = splitmix64(np.arange(n, dtype=np.uint64), _stream_seed(seed, name))
    u = (z >> np.uint64(40)).astype(np.float32) * np.float32(2.0 ** -24)
    return (u * np.float32(2.0) - np.float32(1.0)).astype(np.float32)


def _u(name, shape, seed, lo, hi):
    n = int(np.prod(shape))
    x = uniform(name, n, seed)
    mid, half = np.float32((lo + hi) / 2), np.float32((hi - lo) / 2)
    return (mid + half * x).astype(np.float32).reshape(shape)


def cvit_param_specs(dim=1024, depth=6, mlp_dim=2048, num_classes=2, channels=512, patch_size=7):
    """(name, shape, kind) for every state_dict key, in cvit.py's order."""
    specs = [("pos_embedding", (32, 1, dim), "emb"), ("cls_token", (1, 1, dim), "emb")]
    for (ci, co), (cidx, bidx) in zip(STEM_CHANNELS, stem_module_indices()):
        specs += [(f"features.{cidx}.weight", (co, ci, 3, 3), "conv"),
                  (f"features.{cidx}.bias", (co,), "cbias"),
                  (f"features.{bidx}.weight", (co,), "gamma"),
                  (f"features.{bidx}.bias", (co,), "beta"),
                  (f"features.{bidx}.running_mean", (co,), "rmean"),
                  (f"features.{bidx}.running_var", (co,), "rvar"),
                  (f"features.{bidx}.num_batches_tracked", (), "nbt")]
    pdim = channels * patch_size ** 2
    specs += [("patch_to_embedding.weight", (dim, pdim), "lin"),
              ("patch_to_embedding.bias", (dim,), "lbias")]
    for l in range(depth):
        p = f"transformer.layers.{l}"
        specs += [(f"{p}.0.fn.norm.weight", (dim,), "gamma"),
                  (f"{p}.0.fn.norm.bias", (dim,), "beta"),
                  (f"{p}.0.fn.fn.to_qkv.weight", (3 * dim, dim), "lin"),
                  (f"{p}.0.fn.fn.to_out.weight", (dim, dim), "lin"),
                  (f"{p}.0.fn.fn.to_out.bias", (dim,), "lbias"),
                  (f"{p}.1.fn.norm.weight", (dim,), "gamma"),
                  (f"{p}.1.fn.norm.bias", (dim,), "beta"),
                  (f"{p}.1.fn.fn.net.0.weight", (mlp_dim, dim), "lin"),
                  (f"{p}.1.fn.fn.net.0.bias", (mlp_dim,), "lbias"),
                  (f"{p}.1.fn.fn.net.2.weight", (dim, mlp_dim), "lin"),
                  (f"{p}.1.fn.fn.net.2.bias", (dim,), "lbias")]
    specs += [("mlp_head.0.weight", (mlp_dim, dim), "lin"),
              ("mlp_head.0.bias", (mlp_dim,), "lbias"),
              ("mlp_head.2.weight", (num_classes, mlp_dim), "head"),
              ("mlp_head.2.bias", (num_classes,), "lbias")]
    return specs


def make_state_dict(seed: int = 0, **kw) -> "OrderedDict[str, np.ndarray]":
    """Synthetic CViT state_dict as float32 numpy arrays (int64 for BN counters).

    Scales: He-uniform convs (activations stay O(1) through 17 ReLU layers),
    non-degenerate BN statistics (so a BN-fold bug cannot hide),
    PyTorch-default-bound linears, and a head scaled so logits are O(1) and
    the per-logit sigmoids are not saturated.
    """
    sd = OrderedDict()
    for name, shape, kind in cvit_param_specs(**kw):
        if kind == "nbt":
            sd[name] = np.array(0, dtype=np.int64)
            continue
        if kind == "conv":
            fan_in = shape[1] * shape[2] * shape[3]
            a = float(np.sqrt(6.0 / fan_in))
            sd[name] = _u(name, shape, seed, -a, a)
        elif kind == "lin":
            a = float(1.0 / np.sqrt(shape[1]))
            sd[name] = _u(name, shape, seed, -a, a)
        elif kind == "head":
            a = float(4.0 / np.sqrt(shape[1]))
            sd[name] = _u(name, shape, seed, -a, a)
        elif kind == "emb":
            sd[name] = _u(name, shape, seed, -0.5, 0.5)
        elif kind == "cbias":
            sd[name] = _u(name, shape, seed, -0.05, 0.05)
        elif kind == "lbias":
            sd[name] = _u(name, shape, seed, -0.02, 0.02)
        elif kind == "gamma":
            sd[name] = _u(name, shape, seed, 0.8, 1.2)
        elif kind == "beta":
            sd[name] = _u(name, shape, seed, -0.1, 0.1)
        elif kind == "rmean":
            sd[name] = _u(name, shape, seed, -0.1, 0.1)
        elif kind == "rvar":
            sd[name] = _u(name, shape, seed, 0.8, 1.2)
        else:  # pragma: no cover
            raise ValueError(kind)
    return sd


def make_crops(n: int, seed: int, size: int = 224) -> np.ndarray:
    """n synthetic uint8 NHWC crops [n, size, size, 3], uniform 0..255."""
    z = splitmix64(np.arange(n * size * size * 3, dtype=np.uint64), _stream_seed(seed, "crops"))
    return (z >> np.uint64(56)).astype(np.uint8).reshape(n, size, size, 3)


def state_dict_checksums(sd) -> dict:
    """Per-tensor float64 sum / abs-sum, for pinning the generator in tests."""
    return {k: (float(np.asarray(v, np.float64).sum()), float(np.abs(np.asarray(v, np.float64)).sum()))
            for k, v in sd.items()}


# ---------------------------------------------------------------- ResVitKan
# CViT-main/ResVitKan/ResVitKan.py: resnet50() stem (Bottleneck [3,4,6,3],
# :259-264) + `channel` 1x1 2048->512 + bn2 (:202-203), the CViT embedding /
# transformer (:284-302), kan_head = Linear -> Dropout -> ReLU -> KAN([2048,
# 64, 2]) (:302-307) and the unused mlp_head (:309-314).
RESNET50_LAYERS = [(64, 3, 1), (128, 4, 2), (256, 6, 2), (512, 3, 2)]  # (planes, blocks, stride)
KAN_GRID_SIZE, KAN_ORDER = 5, 3


def resnet50_blocks():
    """(prefix, inplanes, planes, stride, has_downsample) per Bottleneck, in
    _make_layer order (ResVitKan.py:216-230)."""
    out, inplanes = [], 64
    for li, (planes, blocks, stride) in enumerate(RESNET50_LAYERS):
        for b in range(blocks):
            s = stride if b == 0 else 1
            ds = b == 0 and (s != 1 or inplanes != planes * 4)
            out.append((f"features.layer{li + 1}.{b}", inplanes, planes, s, ds))
            inplanes = planes * 4
    return out


def _bn_specs(p, c, gamma_kind="gamma"):
    return [(f"{p}.weight", (c,), gamma_kind), (f"{p}.bias", (c,), "beta"), (f"{p}.running_mean", (c,), "rmean"),
            (f"{p}.running_var", (c,), "rvar"), (f"{p}.num_batches_tracked", (), "nbt")]


def resvitkan_param_specs(dim=1024, depth=6, mlp_dim=2048, num_classes=2, channels=512, patch_size=7):
    """(name, shape, kind) for every key of ResVitKan.CViT's state_dict, in its order (408 keys)."""
    specs = [("pos_embedding", (32, 1, dim), "emb"), ("cls_token", (1, 1, dim), "emb"),
             ("features.conv1.weight", (64, 3, 7, 7), "conv")]
    specs += _bn_specs("features.bn1", 64)
    for p, inp, planes, _s, ds in resnet50_blocks():
        specs += [(f"{p}.conv1.weight", (planes, inp, 1, 1), "conv")] + _bn_specs(f"{p}.bn1", planes)
        specs += [(f"{p}.conv2.weight", (planes, planes, 3, 3), "conv")] + _bn_specs(f"{p}.bn2", planes)
        specs += [(f"{p}.conv3.weight", (planes * 4, planes, 1, 1), "conv")] + _bn_specs(f"{p}.bn3", planes * 4,
                                                                                          "gamma_res")
        if ds:
            specs += [(f"{p}.downsample.0.weight", (planes * 4, inp, 1, 1), "conv")]
            specs += _bn_specs(f"{p}.downsample.1", planes * 4)
    specs += [("features.channel.weight", (channels, 2048, 1, 1), "conv")] + _bn_specs("features.bn2", channels)
    pdim = channels * patch_size ** 2
    specs += [("patch_to_embedding.weight", (dim, pdim), "lin"), ("patch_to_embedding.bias", (dim,), "lbias")]
    specs += [s for s in cvit_param_specs(dim, depth, mlp_dim, num_classes, channels, patch_size)
              if s[0].startswith("transformer.")]
    specs += [("kan_head.0.weight", (mlp_dim, dim), "lin"), ("kan_head.0.bias", (mlp_dim,), "lbias")]
    nb = KAN_GRID_SIZE + KAN_ORDER
    for i, (fi, fo) in enumerate([(mlp_dim, 64), (64, num_classes)]):
        p = f"kan_head.3.layers.{i}"
        specs += [(f"{p}.base_weight", (fo, fi), "kbase"), (f"{p}.spline_weight", (fo, fi, nb), "kspline"),
                  (f"{p}.spline_scaler", (fo, fi), "kscaler"),
                  (f"{p}.grid", (fi, KAN_GRID_SIZE + 2 * KAN_ORDER + 1), "kgrid")]
    specs += [("mlp_head.0.weight", (mlp_dim, dim), "lin"), ("mlp_head.0.bias", (mlp_dim,), "lbias"),
              ("mlp_head.3.weight", (num_classes, mlp_dim), "head"), ("mlp_head.3.bias", (num_classes,), "lbias")]
    return specs


def kan_grid(in_features: int) -> np.ndarray:
    """KANLinear's initial knot buffer (kan.py:39-48): arange(-3, 9) * 0.4 - 1 in float32."""
    h = np.float32((1 - (-1)) / KAN_GRID_SIZE)
    k = np.arange(-KAN_ORDER, KAN_GRID_SIZE + KAN_ORDER + 1).astype(np.float32)
    g = (k * h).astype(np.float32) + np.float32(-1)
    return np.broadcast_to(g.astype(np.float32), (in_features, g.size)).copy()


def make_resvitkan_state_dict(seed: int = 0, **kw) -> "OrderedDict[str, np.ndarray]":
    """Synthetic ResVitKan weights (same scheme as make_state_dict).  The last
    BN of every Bottleneck gets a small gamma (0.1..0.3) so the residual
    stream of 16 blocks stays O(1) (the non-standard ReLU-before-add of
    ResVitKan.py:146-152 only ever adds), and the KAN weights are scaled for
    O(1), unsaturated logits."""
    sd = OrderedDict()
    for name, shape, kind in resvitkan_param_specs(**kw):
        if kind == "nbt":
            sd[name] = np.array(0, dtype=np.int64)
        elif kind == "conv":
            fan_in = int(np.prod(shape[1:]))
            a = float(np.sqrt(6.0 / fan_in))
            sd[name] = _u(name, shape, seed, -a, a)
        elif kind == "gamma_res":
            sd[name] = _u(name, shape, seed, 0.1, 0.3)
        elif kind == "kgrid":
            sd[name] = kan_grid(shape[0])
        elif kind in ("kbase", "kscaler"):
            # the 64 -> 2 layer is scaled up so the logits are O(1)
            a = float((8.0 if ".layers.1." in name else 1.0) / np.sqrt(shape[1]))
            sd[name] = _u(name, shape, seed, -a, a)
        elif kind == "kspline":
            sd[name] = _u(name, shape, seed, -0.5, 0.5)
        else:
            sd[name] = _synthetic(name, shape, kind, seed)
    return sd


def _synthetic(name, shape, kind, seed):
    if kind == "lin":
        a = float(1.0 / np.sqrt(shape[1]))
        return _u(name, shape, seed, -a, a)
    if kind == "head":
        a = float(4.0 / np.sqrt(shape[1]))
        return _u(name, shape, seed, -a, a)
    ranges = {"emb": (-0.5, 0.5), "cbias": (-0.05, 0.05), "lbias": (-0.02, 0.02), "gamma": (0.8, 1.2),
              "beta": (-0.1, 0.1), "rmean": (-0.1, 0.1), "rvar": (0.8, 1.2)}
    lo, hi = ranges[kind]
    return _u(name, shape, seed, lo, hi)


# ---------------------------------------------------------------- S3D
# sx_exp_deepfakedetect-master/S3D/model.py: S3D(num_class, SRM_net) (:6-48)
# with BasicConv3d / SepConv3d (:50-82, BatchNorm3d eps 1e-3) and the
# Mixed_* Inception blocks (:84-342).  Each entry of S3D_BASE is one
# nn.Sequential index of `base`:
#   ("sep", cin, cout, k, stride, pad) | ("basic", cin, cout) | ("pool", k, s, p)
#   | ("mixed", cin, b0, (b1a, b1b), (b2a, b2b), b3)
S3D_MIXED = {
    5: (192, 64, (96, 128), (16, 32), 32), 6: (256, 128, (128, 192), (32, 96), 64),
    8: (480, 192, (96, 208), (16, 48), 64), 9: (512, 160, (112, 224), (24, 64), 64),
    10: (512, 128, (128, 256), (24, 64), 64), 11: (512, 112, (144, 288), (32, 64), 64),
    12: (528, 256, (160, 320), (32, 128), 128), 14: (832, 256, (160, 320), (32, 128), 128),
    15: (832, 384, (192, 384), (48, 128), 128)}
S3D_POOLS = {1: ((1, 3, 3), (1, 2, 2), (0, 1, 1)), 4: ((1, 3, 3), (1, 2, 2), (0, 1, 1)),
             7: ((3, 3, 3), (2, 2, 2), (1, 1, 1)), 13: ((2, 2, 2), (2, 2, 2), (0, 0, 0))}


def s3d_base(srm: bool):
    """The `base` Sequential of S3D (model.py:17-33) as layer descriptors."""
    cin = 30 if srm else 3
    out = []
    for i in range(16):
        if i == 0:
            out.append(("sep", cin, 64, 7, 2, 3))
        elif i == 2:
            out.append(("basic", 64, 64))
        elif i == 3:
            out.append(("sep", 64, 192, 3, 1, 1))
        elif i in S3D_POOLS:
            out.append(("pool",) + S3D_POOLS[i])
        else:
            out.append(("mixed",) + S3D_MIXED[i])
    return out


def _s3d_bn(p, c):
    return [(f"{p}.weight", (c,), "gamma"), (f"{p}.bias", (c,), "beta"), (f"{p}.running_mean", (c,), "rmean"),
            (f"{p}.running_var", (c,), "rvar"), (f"{p}.num_batches_tracked", (), "nbt")]


def _s3d_basic(p, cin, cout):
    return [(f"{p}.conv.weight", (cout, cin, 1, 1, 1), "conv")] + _s3d_bn(f"{p}.bn", cout)


def _s3d_sep(p, cin, cout, k):
    return ([(f"{p}.conv_s.weight", (cout, cin, 1, k, k), "conv")] + _s3d_bn(f"{p}.bn_s", cout) +
            [(f"{p}.conv_t.weight", (cout, cout, k, 1, 1), "conv")] + _s3d_bn(f"{p}.bn_t", cout))


def s3d_param_specs(num_class: int = 1, srm: bool = False):
    """(name, shape, kind) for every key of S3D's state_dict, in its order."""
    specs = [("SRM.hpf.weight", (30, 3, 1, 5, 5), "srm")]
    for i, L in enumerate(s3d_base(srm)):
        p = f"base.{i}"
        if L[0] == "sep":
            specs += _s3d_sep(p, L[1], L[2], L[3])
        elif L[0] == "basic":
            specs += _s3d_basic(p, L[1], L[2])
        elif L[0] == "mixed":
            cin, b0, (b1a, b1b), (b2a, b2b), b3 = L[1:]
            specs += _s3d_basic(f"{p}.branch0.0", cin, b0)
            specs += _s3d_basic(f"{p}.branch1.0", cin, b1a) + _s3d_sep(f"{p}.branch1.1", b1a, b1b, 3)
            specs += _s3d_basic(f"{p}.branch2.0", cin, b2a) + _s3d_sep(f"{p}.branch2.1", b2a, b2b, 3)
            specs += _s3d_basic(f"{p}.branch3.1", cin, b3)
    specs += [("fc.0.weight", (num_class, 1024, 1, 1, 1), "fc"), ("fc.0.bias", (num_class,), "lbias")]
    return specs


def make_s3d_state_dict(seed: int = 0, num_class: int = 1, srm: bool = False) -> "OrderedDict[str, np.ndarray]":
    """Synthetic S3D weights (same scheme as make_state_dict).  Inputs are raw
    0..255 pixels (S3D-test.py:94-96 feeds un-normalised clips), so BN running
    means/vars of the first layer are scaled to that range; the SRM filters
    are zero-sum 5x5 high-pass kernels like the reference bank's."""
    sd = OrderedDict()
    for name, shape, kind in s3d_param_specs(num_class, srm):
        if kind == "nbt":
            sd[name] = np.array(0, dtype=np.int64)
        elif kind == "conv":
            fan_in = int(np.prod(shape[1:]))
            a = float(np.sqrt(6.0 / fan_in))
            sd[name] = _u(name, shape, seed, -a, a)
        elif kind == "srm":
            w = _u(name, shape, seed, -0.25, 0.25)
            w = w - w.mean(axis=(3, 4), keepdims=True)   # high-pass: each 5x5 kernel sums to 0
            sd[name] = w.astype(np.float32)
        elif kind == "fc":
            a = float(4.0 / np.sqrt(shape[1]))
            sd[name] = _u(name, shape, seed, -a, a)
        elif name.startswith("base.0.bn_s.") and kind in ("rmean", "rvar"):
            # first conv sees 0..255 pixels (or SRM residuals of them): BN statistics on that scale
            lo, hi = ((-40.0, 40.0) if kind == "rmean" else (2.0e4, 6.0e4)) if not srm else \
                ((-2.0, 2.0) if kind == "rmean" else (8.0e3, 2.4e4))
            sd[name] = _u(name, shape, seed, lo, hi)
        elif kind == "gamma":
            # ReLU'd activations feed BNs whose synthetic running means are ~0: keep the
            # ~30-layer stack from growing by shrinking every BN scale
            sd[name] = _u(name, shape, seed, 0.8, 1.0)
        else:
            sd[name] = _synthetic(name, shape, kind, seed)
    return sd


def s3d_clips(n: int, frames: int, size: int, seed: int) -> np.ndarray:
    """n synthetic raw clips [n, 3, frames, size, size] float32 of integer pixel
    values 0..255 (S3D's un-normalised BGR input, S3D-test.py:94-96)."""
    z = splitmix64(np.arange(n * 3 * frames * size * size, dtype=np.uint64), _stream_seed(seed, "clips"))
    return (z >> np.uint64(56)).astype(np.float32).reshape(n, 3, frames, size, size)


def s3d_clips_varied(n: int, frames: int, size: int, seed: int) -> np.ndarray:
    """n raw clips [n, 3, frames, size, size] (float32 integers 0..255) that
    differ in content, not only in noise: clip k blends a moving colour
    wave (per-clip direction, speed, phase and brightness; all on a 2^-24
    grid from ``uniform``, so every platform computes the same pixels) with
    uniform noise at weight k/(n-1).  Uniform-noise clips drive every clip to
    almost the same logit; these spread them."""
    p = uniform("clip_params", n * 8, seed).astype(np.float64).reshape(n, 8)
    noise = s3d_clips(n, frames, size, seed).astype(np.float64)
    t = np.arange(frames, dtype=np.float64)[:, None, None] / frames
    yy = np.arange(size, dtype=np.float64)[None, :, None] / size
    xx = np.arange(size, dtype=np.float64)[None, None, :] / size
    out = np.empty((n, 3, frames, size, size), np.float32)
    for k in range(n):
        a, b, c, ph, br, amp = 3 * p[k, 0], 3 * p[k, 1], 2 * p[k, 2], np.pi * p[k, 3], 40 * p[k, 4], 60 + 30 * p[k, 5]
        alpha = k / max(n - 1, 1)
        for ch in range(3):
            wave = 128 + br + amp * np.sin(2 * np.pi * (a * xx + b * yy + c * t) + ph + 2.1 * ch)
            v = (1 - alpha) * wave + alpha * noise[k, ch]
            out[k, ch] = np.clip(np.rint(v), 0, 255)
    return out


# ---------------------------------------------------------------- CViT RepBn8
# CViT-main/model/cvit_GGCA_ADD_DEConv_RepBn8.py::CViT (:343-455): the CViT
# stem with DEConv blocks (:320-340, five parallel 3x3 / 1-D kernels summed
# into one 3x3 at eval), GGCA on the 7x7x512 features (:144-207), attention
# PreNorm = LayerNorm(eps 1e-5), FeedForward PreNorm = LinearNorm, whose eval
# path is LayerNorm(eps 1e-6) (:22-46).  One entry per conv of features1 /
# features2 (nn.Sequential indices):
#   (sequential, index, kind "conv" | "deconv", cin, cout, bn index | None, relu, pool after)
REPBN8_LAYERS = [
    ("features1", 0, "conv", 3, 32, 1, True, False),
    ("features1", 3, "deconv", 32, 32, 4, True, False),
    ("features1", 6, "deconv", 32, 32, 7, True, True),
    ("features1", 10, "conv", 32, 64, 11, True, False),
    ("features1", 13, "deconv", 64, 64, 14, True, False),
    ("features1", 16, "deconv", 64, 64, 17, True, True),
    ("features1", 20, "conv", 64, 128, 21, True, False),
    ("features1", 23, "deconv", 128, 128, 24, True, False),
    ("features1", 26, "conv", 128, 128, None, False, False),   # :390 Conv2d(128,128) - no BN, no ReLU
    ("features1", 27, "deconv", 128, 128, None, True, True),   # :391-392 DEConv(128) -> ReLU
    ("features1", 30, "conv", 128, 256, 31, True, False),
    ("features1", 33, "deconv", 256, 256, 34, True, False),
    ("features1", 36, "deconv", 256, 256, 37, True, False),
    ("features1", 39, "deconv", 256, 256, 40, True, True),
    ("features2", 0, "conv", 256, 512, 1, True, False),
    ("features2", 3, "deconv", 512, 512, 4, True, False),
    ("features2", 6, "deconv", 512, 512, 7, True, False),
    ("features2", 9, "deconv", 512, 512, 10, True, True),
]
DECONV_PARTS = ("conv1_1.conv", "conv1_2.conv", "conv1_3.conv", "conv1_4.conv", "conv1_5")


def _deconv_specs(p, c):
    out = []
    for part in DECONV_PARTS:
        shape = (c, c, 3) if part in ("conv1_2.conv", "conv1_3.conv") else (c, c, 3, 3)
        out += [(f"{p}.{part}.weight", shape, "dconv"), (f"{p}.{part}.bias", (c,), "cbias")]
    return out


def repbn8_param_specs(dim=1024, depth=6, mlp_dim=2048, num_classes=2, channels=512, patch_size=7):
    """(name, shape, kind) for every key of the RepBn8 CViT's state_dict, in its order."""
    specs = [("pos_embedding", (32, 1, dim), "emb"), ("cls_token", (1, 1, dim), "emb")]
    for seq, idx, kind, ci, co, bn, _relu, _pool in REPBN8_LAYERS:
        p = f"{seq}.{idx}"
        if kind == "conv":
            specs += [(f"{p}.weight", (co, ci, 3, 3), "conv"), (f"{p}.bias", (co,), "cbias")]
        else:
            specs += _deconv_specs(p, co)
        if bn is not None:
            specs += _bn_specs(f"{seq}.{bn}", co)
    pdim = channels * patch_size ** 2
    specs += [("patch_to_embedding.weight", (dim, pdim), "lin"), ("patch_to_embedding.bias", (dim,), "lbias")]
    for l in range(depth):
        p = f"transformer.layers.{l}"
        specs += [(f"{p}.0.fn.norm.weight", (dim,), "gamma"), (f"{p}.0.fn.norm.bias", (dim,), "beta"),
                  (f"{p}.0.fn.fn.to_qkv.weight", (3 * dim, dim), "lin"),
                  (f"{p}.0.fn.fn.to_out.weight", (dim, dim), "lin"), (f"{p}.0.fn.fn.to_out.bias", (dim,), "lbias"),
                  (f"{p}.1.fn.norm.warm", (), "warm"), (f"{p}.1.fn.norm.iter", (), "step"),
                  (f"{p}.1.fn.norm.total_step", (), "step"),
                  (f"{p}.1.fn.norm.norm1.weight", (dim,), "gamma"), (f"{p}.1.fn.norm.norm1.bias", (dim,), "beta"),
                  (f"{p}.1.fn.norm.norm2.alpha", (1,), "alpha")]
        specs += _bn_specs(f"{p}.1.fn.norm.norm2.bn", dim)
        specs += [(f"{p}.1.fn.fn.net.0.weight", (mlp_dim, dim), "lin"), (f"{p}.1.fn.fn.net.0.bias", (mlp_dim,), "lbias"),
                  (f"{p}.1.fn.fn.net.2.weight", (dim, mlp_dim), "lin"), (f"{p}.1.fn.fn.net.2.bias", (dim,), "lbias")]
    specs += [("mlp_head.0.weight", (mlp_dim, dim), "lin"), ("mlp_head.0.bias", (mlp_dim,), "lbias"),
              ("mlp_head.2.weight", (num_classes, mlp_dim), "head"), ("mlp_head.2.bias", (num_classes,), "lbias")]
    gc = channels // 4                      # GGCA(512, 7, 7): 4 groups, reduction 16 (:144-172)
    specs += [("ggca.shared_conv.0.weight", (gc // 16, gc, 1, 1), "conv"), ("ggca.shared_conv.0.bias", (gc // 16,), "cbias")]
    specs += _bn_specs("ggca.shared_conv.1", gc // 16)
    specs += [("ggca.shared_conv.3.weight", (gc, gc // 16, 1, 1), "conv"), ("ggca.shared_conv.3.bias", (gc,), "cbias")]
    specs += _deconv_specs("Deconv", 256)   # self.Deconv = DEConv(256) (:454): in the state_dict, never called
    return specs


def make_repbn8_state_dict(seed: int = 0, **kw) -> "OrderedDict[str, np.ndarray]":
    """Synthetic RepBn8 weights (same generator).  The five DEConv kernels are
    drawn at 1/2.8 of the He bound each: their folded sum (with the central-
    and angular-difference terms) then has about unit gain, so the features
    stay O(1) through 14 DEConvs (mean |features2| 0.88); LinearNorm's counters are the reference's defaults
    (warm 0, iter = total_step = 300000) and RepBN (unused at eval) is a
    plain alpha = 1 / unit BatchNorm."""
    sd = OrderedDict()
    for name, shape, kind in repbn8_param_specs(**kw):
        if kind == "nbt" or kind == "warm":
            sd[name] = np.array(0, dtype=np.int64)
        elif kind == "step":
            sd[name] = np.array(300000, dtype=np.int64)
        elif kind == "alpha":
            sd[name] = np.ones(shape, dtype=np.float32)
        elif kind in ("conv", "dconv"):
            fan_in = int(np.prod(shape[1:]))
            a = float(np.sqrt(6.0 / fan_in))
            if kind == "dconv":
                a /= 2.8
            sd[name] = _u(name, shape, seed, -a, a)
        else:
            sd[name] = _synthetic(name, shape, kind, seed)
    return sd
