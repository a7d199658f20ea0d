"""Drop-in ``ResVitKan`` (BASELINE config 5) on gfx950 HIP kernels.

Mirrors ``CViT-main/ResVitKan/ResVitKan.py::CViT`` (:284-329): the same
constructor, the same 408-key ``state_dict`` (names, shapes, order — the
``resnet50()`` stem, embedding, transformer, ``kan_head`` and the unused
``mlp_head``) and ``forward(img, mask=None)`` on a normalised fp32 NCHW
``[B,3,224,224]`` batch returning fp32 logits ``[B,2]`` (eval mode: Dropout is
the identity), with the reference's batch-slot ``pos_embedding`` rule.

Arithmetic (no CPU fallback, every layer is a HIP kernel of libfac_cvit.so):

* ResNet-50 stem: each conv + eval BatchNorm (folded on the host in fp32,
  weights rounded once to 16 bits) is one ``fac_conv_nd`` implicit-GEMM launch
  (fac_fake_amd/csrc/ops.hip); the Bottleneck's conv3 epilogue applies bn3,
  ReLU, the residual add and the second ReLU in fp32 (ResVitKan.py:146-152);
  the 3x3/2 max-pool is ``fac_pool_nd``.  Activations are 16-bit NHWC.
* ``channel`` 1x1 + bn2 -> features [B,7,7,512] NHWC, which is already the
  ``(p1 p2 c)`` flatten of ResVitKan.py:320, handed to the CViT tail
  (``fac_forward_features``: patch embedding, cls/pos, 6-layer transformer,
  ``kan_head.0`` + ReLU) — the CViT kernels, loaded "tail_only".
* ``KAN([2048, 64, 2])``: two ``fac_kan_linear`` launches in fp32.

The whole forward can be captured into a hipGraph (``torch.cuda.graph``):
every launch goes to the current torch stream, workspaces come from torch's
caching allocator.
"""
from __future__ import annotations

import ctypes
import math

import torch
from torch import nn

from . import _lib
from .cvit import MAX_SLOTS, _Node, reference_mask_poisons, weight_versions
from .ops import (TORCH16, ConvLayer, KANLinearLayer, bottleneck_pw2, conv_dual, fold_bn, pack_input_s2d,
                  pool, s2d_weight, sigmoid)
from .weights import kan_grid, resnet50_blocks, resvitkan_param_specs

SUPPORTED = dict(image_size=224, patch_size=7, num_classes=2, channels=512, dim=1024, depth=6, heads=8,
                 mlp_dim=2048)
BN_EPS = 1e-5
MEAN = (0.485, 0.456, 0.406)     # helpers/loader.py:9 (the training normalisation)
STD = (0.229, 0.224, 0.225)
_BUFFERS = ("rmean", "rvar", "nbt", "kgrid")


def _init_tensor(name, shape, kind):
    if kind == "nbt":
        return torch.zeros((), dtype=torch.long)
    if kind in ("rmean", "beta", "lbias"):
        return torch.zeros(shape)
    if kind in ("rvar", "gamma", "gamma_res"):
        return torch.ones(shape)
    if kind == "emb":
        return torch.randn(shape)
    if kind == "kgrid":
        return torch.from_numpy(kan_grid(shape[0]))
    t = torch.empty(shape)
    fan_in = int(math.prod(shape[1:]))
    if kind == "conv":
        return t.normal_(0, math.sqrt(2.0 / fan_in))
    bound = 1.0 / math.sqrt(shape[1] if len(shape) > 1 else 1)
    return t.uniform_(-bound, bound)


class ResVitKan(nn.Module):
    def __init__(self, image_size=224, patch_size=7, num_classes=2, channels=512, dim=1024, depth=6, heads=8,
                 mlp_dim=2048, *, dtype: str = "fp16"):
        super().__init__()
        cfg = dict(image_size=image_size, patch_size=patch_size, num_classes=num_classes, channels=channels, dim=dim,
                   depth=depth, heads=heads, mlp_dim=mlp_dim)
        if cfg != SUPPORTED:
            raise NotImplementedError(f"the gfx950 ResVitKan path implements {SUPPORTED}, got {cfg}")
        if dtype not in _lib.DTYPES:
            raise ValueError(f"dtype must be one of {list(_lib.DTYPES)}")
        self.dtype_name = dtype
        self.patch_size = patch_size
        for name, shape, kind in resvitkan_param_specs(dim=dim, depth=depth, mlp_dim=mlp_dim,
                                                       num_classes=num_classes, channels=channels,
                                                       patch_size=patch_size):
            *path, leaf = name.split(".")
            mod = self
            for p in path:
                if p not in mod._modules:
                    mod.add_module(p, _Node())
                mod = mod._modules[p]
            t = _init_tensor(name, shape, kind)
            if kind in _BUFFERS:
                mod.register_buffer(leaf, t)
            else:
                mod.register_parameter(leaf, nn.Parameter(t))
        self._prep = None          # (device index, versions) the packed layers belong to
        self._ctx = None
        self.eval()

    # ------------------------------------------------------------------ weights
    def _versions(self):
        return weight_versions(self)

    def load_state_dict(self, state_dict, strict: bool = True, assign: bool = False):
        out = super().load_state_dict(state_dict, strict=strict, assign=assign)
        self._prep = None
        return out

    def train(self, mode: bool = True):
        if mode:
            raise RuntimeError("the gfx950 ResVitKan path is inference-only (BatchNorm is folded into the convs)")
        return super().train(False)

    def _release(self):
        if self._ctx is not None:
            _lib.load().fac_destroy(self._ctx)
            self._ctx = None

    def __del__(self):
        try:
            self._release()
        except Exception:
            pass

    def _prepare(self, device: torch.device):
        idx = device.index if device.index is not None else torch.cuda.current_device()
        v = self._versions()
        if self._prep == (idx, v):
            return
        sd = self.state_dict()
        dt = self.dtype_name

        def conv(ck, bnp, stride=1, pad=0, cin_pad=None):
            w, b = fold_bn(sd[ck], None, sd[bnp + ".weight"], sd[bnp + ".bias"], sd[bnp + ".running_mean"],
                           sd[bnp + ".running_var"], BN_EPS)
            return ConvLayer(w, b, stride, pad, dtype=dt, device=device, cin_pad=cin_pad)

        # conv1 7x7/2 (3 channels) as a 4x4/1 conv over space-to-depth cells (ops.s2d_weight)
        w1, b1 = fold_bn(sd["features.conv1.weight"], None, sd["features.bn1.weight"], sd["features.bn1.bias"],
                         sd["features.bn1.running_mean"], sd["features.bn1.running_var"], BN_EPS)
        self._conv1 = ConvLayer(s2d_weight(w1), b1, 1, 0, dtype=dt, device=device)
        self._blocks = []
        for p, _inp, _planes, s, ds in resnet50_blocks():
            self._blocks.append((conv(p + ".conv1.weight", p + ".bn1"),
                                 conv(p + ".conv2.weight", p + ".bn2", s, 1),
                                 conv(p + ".conv3.weight", p + ".bn3"),
                                 conv(p + ".downsample.0.weight", p + ".downsample.1", s) if ds else None))
        self._channel = conv("features.channel.weight", "features.bn2")
        self._kan = [KANLinearLayer(sd[f"kan_head.3.layers.{i}.grid"], sd[f"kan_head.3.layers.{i}.base_weight"],
                                    sd[f"kan_head.3.layers.{i}.spline_weight"],
                                    sd[f"kan_head.3.layers.{i}.spline_scaler"], device) for i in range(2)]
        # the CViT tail (embedding .. first head layer), loaded without a conv stem
        lib = _lib.load()
        self._release()
        h = ctypes.c_void_p()
        _lib.check(lib.fac_create(idx, _lib.DTYPES[dt], ctypes.byref(h)), None, "fac_create")
        self._ctx = h
        _lib.check(lib.fac_set_option(h, b"tail_only", 1), h, "fac_set_option")
        tail = {k: t for k, t in sd.items() if k in ("pos_embedding", "cls_token") or
                k.startswith("patch_to_embedding.") or k.startswith("transformer.")}
        tail["mlp_head.0.weight"] = sd["kan_head.0.weight"]
        tail["mlp_head.0.bias"] = sd["kan_head.0.bias"]
        tail["mlp_head.2.weight"] = torch.zeros(2, sd["kan_head.0.weight"].shape[0])  # unused: logits come from the KAN
        tail["mlp_head.2.bias"] = torch.zeros(2)
        keep, descs = [], []
        for k, t in tail.items():
            hst = t.detach().to("cpu", torch.float32).contiguous()
            keep.append(hst)
            d = _lib.TensorDesc()
            d.name, d.data, d.ndim = k.encode(), hst.data_ptr(), hst.dim()
            for i, s in enumerate(hst.shape):
                d.shape[i] = s
            descs.append(d)
        arr = (_lib.TensorDesc * len(descs))(*descs)
        _lib.check(lib.fac_load_weights(h, ctypes.cast(arr, ctypes.c_void_p), len(descs)), h, "fac_load_weights")
        self._prep = (idx, v)

    def reserve(self, max_batch: int, device=None):
        dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        self._prepare(dev)
        _lib.check(_lib.load().fac_reserve(self._ctx, int(max_batch)), self._ctx, "fac_reserve")

    # ------------------------------------------------------------------ forward
    # crops per pass of the ResNet stem (0 = the whole batch).  Smaller chunks
    # keep a block's activations in the Infinity Cache, but measured on MI355X
    # (B = 256, bf16) the whole batch is fastest: 8.9 ms vs 9.5 / 11.0 / 15.6
    # ms at 128 / 64 / 32 — the layers are not HBM-bound, the smaller grids
    # just fill the 256 CUs worse (tools/archive/rvk_chunks.sh)
    feature_chunk = 0
    # a layer1 bottleneck's conv3 and the next block's conv1 run as one launch
    # (fac_bottleneck_pw2).  Layer2's pairs stay two launches: the fused
    # layer2 kernel (bneck_pw2_l2) is correct but measured slower (69.3k vs
    # 69.7-69.9k crops/s same box).

    @staticmethod
    def _pw2_ok(c3, c1n, x) -> bool:
        """fac_bottleneck_pw2's shapes: conv3 1x1 64 -> 256, the next conv1 1x1
        256 -> 64 / 128 at stride 1 (torchvision v1.5 puts the stride on conv2)."""
        g3, g1 = c3.g, c1n.g
        shapes = c3.cin == 64 and c3.cout == 256 and c1n.cin == 256 and c1n.cout in (64, 128)
        return (shapes and (g3.kd, g3.kh, g3.kw, g3.sd, g3.sh, g3.sw) == (1,) * 6
                and (g1.kd, g1.kh, g1.kw, g1.sd, g1.sh, g1.sw) == (1,) * 6
                and (g1.pd, g1.ph, g1.pw) == (0, 0, 0) and x.shape[-1] == c3.cout)

    def features16(self, x16: torch.Tensor, out: torch.Tensor | None = None, taps: list | None = None) -> torch.Tensor:
        """ResNet.forward (ResVitKan.py:232-247) on space-to-depth packed 16-bit
        cells [B,1,115,115,16] (ops.pack_input_s2d) -> [B,1,7,7,512] 16-bit
        NHWC, in chunks of ``feature_chunk`` crops.  With `taps` (one chunk
        only): the max-pool output, every Bottleneck's output and the bn2
        output, [B,1,H,W,C] 16-bit, are appended to it."""
        B = x16.shape[0]
        if out is None:
            out = torch.empty(B, 1, 7, 7, 512, dtype=x16.dtype, device=x16.device)
        step = B if taps is not None else (self.feature_chunk or B)
        tap = taps.append if taps is not None else (lambda t: None)
        for b0 in range(0, B, step):
            # 7x7/2 + bn1 + ReLU + MaxPool2d(3, 2, 1) in one launch (conv_s2d4_mp)
            x = self._conv1(x16[b0:b0 + step], maxpool3s2=True)
            tap(x)
            h1 = None  # the next block's conv1 output, when the previous conv3 computed it
            for bi, (c1, c2, c3, ds) in enumerate(self._blocks):
                nxt = self._blocks[bi + 1] if bi + 1 < len(self._blocks) else None
                if ds is None and nxt is not None and self._pw2_ok(c3, nxt[0], x):
                    # conv3 (+ identity residual) and the next block's conv1 in
                    # one launch (fac_bottleneck_pw2): x is not read back
                    x, h1n = bottleneck_pw2(c3, c2(h1 if h1 is not None else c1(x)), x, nxt[0])
                    h1 = h1n
                    tap(x)
                    continue
                if ds is not None:
                    # conv3 + bn3 + ReLU and the downsample conv + bn in one launch
                    # (fac_conv_nd_dual): the residual never goes through memory
                    x = conv_dual(c3, c2(h1 if h1 is not None else c1(x)), ds, x)
                    h1 = None
                    tap(x)
                    continue
                res = x
                h = c2(h1 if h1 is not None else c1(x))
                h1 = None
                x = c3(h, residual=res, relu2=True)                 # relu(bn3) + residual, relu
                tap(x)
            self._channel(x, relu=False, out=out[b0:b0 + step])     # channel 1x1 + bn2
            tap(out[b0:b0 + step])
        return out

    def stage_outputs(self, crops: torch.Tensor) -> list:
        """For uint8 crops [B,224,224,3]: the ResNet-50 outputs a forward hook on
        the reference's ``features.maxpool``, each ``features.layerN[b]`` and
        ``features.bn2`` sees (18 tensors, NHWC 16-bit), for per-block parity."""
        if crops.dtype != torch.uint8 or crops.dim() != 4 or tuple(crops.shape[1:]) != (224, 224, 3):
            raise ValueError(f"expected uint8 crops [B,224,224,3], got {crops.dtype} {tuple(crops.shape)}")
        if not crops.is_cuda:
            raise RuntimeError("ResVitKan (gfx950 HIP path) needs its input on a GPU device; there is no CPU fallback")
        self._prepare(crops.device)
        x16 = pack_input_s2d(crops, dtype=self.dtype_name, u8=True, div=255.0, mean=MEAN, std=STD)
        taps = []
        self.features16(x16, taps=taps)
        return taps

    def _run(self, x16: torch.Tensor, pos_index, want_probs: bool):
        B = x16.shape[0]
        dev = x16.device
        pidx = _pos_index(B, pos_index, dev)
        f = self.features16(x16)
        hidden = torch.empty(B, SUPPORTED["mlp_dim"], dtype=torch.float32, device=dev)
        lib = _lib.load()
        _lib.check(lib.fac_forward_features(self._ctx, f.data_ptr(), B, pidx.data_ptr(), hidden.data_ptr(), None,
                                            None, torch.cuda.current_stream(dev).cuda_stream), self._ctx,
                   "fac_forward_features")
        logits = self._kan[1](self._kan[0](hidden))
        return logits, (sigmoid(logits) if want_probs else None)

    def forward(self, img: torch.Tensor, mask=None, pos_index=None) -> torch.Tensor:
        poison = mask is not None and reference_mask_poisons(mask, img.shape[0])
        if not img.is_cuda:
            raise RuntimeError("ResVitKan (gfx950 HIP path) needs its input on a GPU device; there is no CPU fallback")
        if img.dim() != 4 or tuple(img.shape[1:]) != (3, 224, 224):
            raise ValueError(f"expected img [B,3,224,224], got {tuple(img.shape)}")
        self._prepare(img.device)
        x16 = pack_input_s2d(img.float(), dtype=self.dtype_name, u8=False)
        logits = self._run(x16, pos_index, False)[0]
        return logits.fill_(float("nan")) if poison else logits

    def forward_u8(self, crops: torch.Tensor, pos_index=None, return_probs: bool = False):
        """uint8 NHWC RGB crops [B,224,224,3]; x/255 + ImageNet Normalize fused into the input packing."""
        if crops.dtype != torch.uint8 or crops.dim() != 4 or tuple(crops.shape[1:]) != (224, 224, 3):
            raise ValueError(f"expected uint8 crops [B,224,224,3], got {crops.dtype} {tuple(crops.shape)}")
        if not crops.is_cuda:
            raise RuntimeError("ResVitKan (gfx950 HIP path) needs its input on a GPU device; there is no CPU fallback")
        self._prepare(crops.device)
        x16 = pack_input_s2d(crops, dtype=self.dtype_name, u8=True, div=255.0, mean=MEAN, std=STD)
        logits, probs = self._run(x16, pos_index, return_probs)
        return (logits, probs) if return_probs else logits


def _pos_index(B: int, pos_index, device) -> torch.Tensor:
    if pos_index is None:
        if B > MAX_SLOTS:   # `x += self.pos_embedding[0:shape]` (ResVitKan.py:324-325) raises past 32
            raise RuntimeError(f"The size of tensor a ({B}) must match the size of tensor b ({MAX_SLOTS}) "
                               f"at non-singleton dimension 0")
        return torch.arange(B, dtype=torch.int32, device=device)
    p = torch.as_tensor(pos_index)
    if p.shape != (B,):
        raise ValueError(f"pos_index must have shape ({B},), got {tuple(p.shape)}")
    # (a device tensor is range-checked eagerly, not while a hipGraph is being captured)
    if p.numel() and not torch.cuda.is_current_stream_capturing() and (int(p.min()) < 0 or int(p.max()) >= MAX_SLOTS):
        raise IndexError(f"pos_index values must lie in [0, {MAX_SLOTS})")
    return p.to(device=device, dtype=torch.int32).contiguous()


__all__ = ["ResVitKan", "TORCH16"]
