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
