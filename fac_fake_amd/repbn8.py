"""Drop-in CViT RepBn8 variant on gfx950 HIP kernels.

Mirrors ``CViT-main/model/cvit_GGCA_ADD_DEConv_RepBn8.py::CViT`` (:343-455),
the variant most of the reference's recorded predictions come from
(``wprediction/4090RepBn8_*.csv``): the same constructor, the same 359-key
``state_dict`` (names, shapes, order — DEConv's five kernels, GGCA,
LinearNorm's counters and its unused RepBN branch, the unused top-level
``Deconv``) and ``forward(img, mask=None)`` on a normalised fp32 NCHW
``[B,3,224,224]`` batch returning fp32 logits ``[B,2]`` in eval mode, with
the reference's batch-slot ``pos_embedding`` rule.

Arithmetic (no CPU fallback, every layer is a HIP kernel of libfac_cvit.so):

* The 18 convs of ``features1`` / ``features2`` run on the CViT's own
  conv-stack kernels: each DEConv (:320-340) is folded on the host at load
  time into the single 3x3 kernel its eval forward convolves with
  (``deconv_fold``, the reference's weight algebra in its op order, fp32),
  eval BatchNorm is folded on top; the first block (conv, DEConv, DEConv,
  pool — the CViT's conv1-3 shape) is the fused ``fac_stem224`` kernel with
  the input normalisation, every later conv one ``fac_conv3x3`` launch
  (halo-staged implicit GEMM, 16-bit NHWC, fp32 accumulation, the 2x2
  max-pool and the ReLU in its epilogue — no ReLU after ``features1.26``,
  :390-392).
* ``x = x * GGCA(x)`` (:144-207, :436-437) is one ``fac_ggca`` launch.
* Patch embedding, cls/pos, the transformer and the head are the CViT tail
  kernels (``fac_forward_features`` on a "tail_only" context); the
  FeedForward PreNorm is LinearNorm, whose eval branch is LayerNorm(eps 1e-6)
  (:22-48), set with the context option ``ffn_ln_eps_exp`` = 6.

The whole forward is stream-ordered on the current torch stream and can be
captured into a hipGraph.
"""
from __future__ import annotations

import ctypes

import torch
from torch import nn

from . import _lib
from .cvit import MAX_SLOTS, _Node, reference_mask_poisons, weight_versions
from .ops import TORCH16, fold_bn, sigmoid
from .weights import REPBN8_LAYERS, repbn8_param_specs

SUPPORTED = dict(image_size=224, patch_size=7, num_classes=2, channels=512, dim=1024, depth=6, heads=8,
                 mlp_dim=2048)
BN_EPS = 1e-5
FF_LN_EPS_EXP = 6                 # LinearNorm.norm1 = LayerNorm(eps=1e-6) (:48)
_BUFFERS = ("rmean", "rvar", "nbt", "warm", "step")


def deconv_fold(sd, p: str):
    """DEConv.forward's effective 3x3 weight and bias (:329-338): the sum of
    Conv2d_cd (:221-228), Conv2d_hd (:292-297), Conv2d_vd (:310-315),
    Conv2d_ad with theta 1 (:242-246) and the plain conv1_5, evaluated with
    the reference's tensor ops in its order, in fp32 on the CPU."""
    f = lambda k: sd[f"{p}.{k}"].detach().to("cpu", torch.float32)  # noqa: E731
    w1 = f("conv1_1.conv.weight")
    o, i = w1.shape[:2]
    t = w1.reshape(o, i, 9)
    cd = torch.zeros(o, i, 9)
    cd[:, :, :] = t[:, :, :]
    cd[:, :, 4] = t[:, :, 4] - t[:, :, :].sum(2)
    h = f("conv1_2.conv.weight")
    hd = torch.zeros(o, i, 9)
    hd[:, :, [0, 3, 6]] = h[:, :, :]
    hd[:, :, [2, 5, 8]] = -h[:, :, :]
    v = f("conv1_3.conv.weight")
    vd = torch.zeros(o, i, 9)
    vd[:, :, [0, 1, 2]] = v[:, :, :]
    vd[:, :, [6, 7, 8]] = -v[:, :, :]
    a = f("conv1_4.conv.weight").reshape(o, i, 9)
    ad = a - 1.0 * a[:, :, [3, 0, 1, 6, 4, 2, 7, 8, 5]]
    w = (cd.reshape(o, i, 3, 3) + hd.reshape(o, i, 3, 3) + vd.reshape(o, i, 3, 3) + ad.reshape(o, i, 3, 3)
         + f("conv1_5.weight"))
    b = f("conv1_1.conv.bias") + f("conv1_2.conv.bias") + f("conv1_3.conv.bias") + f("conv1_4.conv.bias") + \
        f("conv1_5.bias")
    return w, b


def _init_tensor(shape, kind):
    if kind in ("nbt", "warm"):
        return torch.zeros((), dtype=torch.long)
    if kind == "step":
        return torch.tensor(300000)
    if kind in ("rmean", "beta", "lbias", "cbias"):
        return torch.zeros(shape)
    if kind in ("rvar", "gamma", "alpha"):
        return torch.ones(shape)
    if kind == "emb":
        return torch.randn(shape)
    t = torch.empty(shape)
    fan_in = 1
    for s in shape[1:]:
        fan_in *= s
    return t.uniform_(-1.0 / fan_in ** 0.5, 1.0 / fan_in ** 0.5)


class CViT(nn.Module):
    """cvit_GGCA_ADD_DEConv_RepBn8.CViT on gfx950 (inference)."""

    def __init__(self, image_size=224, patch_size=7, num_classes=2, channels=512, dim=1024, depth=6, heads=8,
                 mlp_dim=2048, *, dtype: str = "fp16"):
        super().__init__()
        cfg = dict(image_size=image_size, patch_size=patch_size, num_classes=num_classes, channels=channels, dim=dim,
                   depth=depth, heads=heads, mlp_dim=mlp_dim)
        if cfg != SUPPORTED:
            raise NotImplementedError(f"the gfx950 RepBn8 path implements {SUPPORTED}, got {cfg}")
        if dtype not in _lib.DTYPES:
            raise ValueError(f"dtype must be one of {list(_lib.DTYPES)}")
        self.dtype_name = dtype
        self.patch_size = patch_size
        for name, shape, kind in repbn8_param_specs(dim=dim, depth=depth, mlp_dim=mlp_dim, num_classes=num_classes,
                                                    channels=channels, patch_size=patch_size):
            *path, leaf = name.split(".")
            mod = self
            for p in path:
                if p not in mod._modules:
                    mod.add_module(p, _Node())
                mod = mod._modules[p]
            t = _init_tensor(shape, kind)
            if kind in _BUFFERS:
                mod.register_buffer(leaf, t)
            else:
                mod.register_parameter(leaf, nn.Parameter(t))
        self._prep = None
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
            raise RuntimeError("the gfx950 RepBn8 path is inference-only (DEConv and BatchNorm are folded)")
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

    def folded_layers(self):
        """(weight, bias, relu, pool) per conv, DEConv and BatchNorm folded in fp32."""
        sd = self.state_dict()
        out = []
        for seq, idx, kind, _ci, _co, bn, relu, pl in REPBN8_LAYERS:
            p = f"{seq}.{idx}"
            w, b = (sd[p + ".weight"], sd[p + ".bias"]) if kind == "conv" else deconv_fold(sd, p)
            if bn is not None:
                q = f"{seq}.{bn}"
                w, b = fold_bn(w, b, sd[q + ".weight"], sd[q + ".bias"], sd[q + ".running_mean"],
                               sd[q + ".running_var"], BN_EPS)
            else:
                w, b = fold_bn(w, b, None, None, None, None, BN_EPS)
            out.append((w, b, relu, pl))
        return out

    def _prepare(self, device: torch.device):
        idx = device.index if device.index is not None else torch.cuda.current_device()
        v = self._versions()
        if self._prep == (idx, v):
            return
        sd = self.state_dict()
        dt = self.dtype_name
        lib = _lib.load()
        dti = _lib.DTYPES[dt]

        def packed(w, H):
            co, ci = w.shape[:2]
            wf = w.reshape(co, ci, 9).contiguous()
            if H == 0:   # the fused block's conv 3->32
                out = torch.empty(32 * 64, dtype=torch.int16)
                _lib.check(lib.fac_stem224_pack_conv1(dti, wf.data_ptr(), out.data_ptr()), None, "pack_conv1")
            else:
                n = lib.fac_conv3x3_packed_elems(H, ci, co)
                if n == 0:
                    raise ValueError(f"conv {ci}->{co} at {H}x{H} is not a fac_conv3x3 shape")
                out = torch.empty(n, dtype=torch.int16)
                _lib.check(lib.fac_conv3x3_pack(dti, H, ci, co, wf.data_ptr(), out.data_ptr()), None, "pack_conv3x3")
            return out.view(TORCH16[dt]).to(device)

        layers, H = [], 224
        for i, (w, b, relu, pl) in enumerate(self.folded_layers()):
            co, ci = w.shape[:2]
            layers.append((packed(w, 0 if i == 0 else H), b.to(device), H, ci, co, pl, relu))
            if pl:
                H //= 2
        (w1, b1, *_), (w2, b2, *_), (w3, b3, *_) = layers[:3]
        self._stem = (w1, b1, w2, b2, w3, b3)
        self._layers = layers[3:]
        self._zero = torch.zeros(128, dtype=torch.int16, device=device)   # zero-padding source page
        g = "ggca.shared_conv."
        f32 = lambda t: t.detach().to(device=device, dtype=torch.float32).contiguous()  # noqa: E731
        cr, cg = sd[g + "0.weight"].shape[:2]
        self._ggca = (f32(sd[g + "0.weight"].reshape(cr, cg)), f32(sd[g + "0.bias"]),
                      f32(torch.stack([sd[g + "1.running_mean"], sd[g + "1.running_var"], sd[g + "1.weight"],
                                       sd[g + "1.bias"]])),
                      f32(sd[g + "3.weight"].reshape(cg, cr)), f32(sd[g + "3.bias"]))
        # the CViT tail (embedding .. head) on a context without a conv stem; the
        # FeedForward PreNorm's LayerNorm is LinearNorm.norm1 (eval branch, :40-41)
        self._release()
        h = ctypes.c_void_p()
        _lib.check(lib.fac_create(idx, _lib.DTYPES[dt], ctypes.byref(h)), None, "fac_create")
        self._ctx = h
        _lib.check(lib.fac_set_option(h, b"tail_only", 1), h, "fac_set_option")
        _lib.check(lib.fac_set_option(h, b"ffn_ln_eps_exp", FF_LN_EPS_EXP), h, "fac_set_option")
        tail = {}
        for k, t in sd.items():
            if k in ("pos_embedding", "cls_token") or k.startswith("patch_to_embedding.") or \
                    k.startswith("mlp_head."):
                tail[k] = t
            elif k.startswith("transformer."):
                if ".1.fn.norm.norm1." in k:
                    tail[k.replace(".norm.norm1.", ".norm.")] = t
                elif ".1.fn.norm." not in k:
                    tail[k] = t
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
    def features(self, src: torch.Tensor, u8: bool) -> torch.Tensor:
        """features1 + features2 (:432-435) -> [B,7,7,512] 16-bit NHWC.  src:
        uint8 NHWC crops (u8) or normalised fp32 NCHW images."""
        lib = _lib.load()
        dti = _lib.DTYPES[self.dtype_name]
        B, dev = src.shape[0], src.device
        st = torch.cuda.current_stream(dev).cuda_stream
        x = torch.empty(B, 112, 112, 32, dtype=TORCH16[self.dtype_name], device=dev)
        w1, b1, w2, b2, w3, b3 = self._stem
        _lib.check(lib.fac_stem224(dti, int(u8), src.data_ptr(), w1.data_ptr(), b1.data_ptr(), w2.data_ptr(),
                                   b2.data_ptr(), w3.data_ptr(), b3.data_ptr(), x.data_ptr(), B, st), None,
                   "fac_stem224")
        for wpk, b, H, ci, co, pl, relu in self._layers:
            Ho = H // 2 if pl else H
            y = torch.empty(B, Ho, Ho, co, dtype=x.dtype, device=dev)
            _lib.check(lib.fac_conv3x3(dti, x.data_ptr(), wpk.data_ptr(), b.data_ptr(), y.data_ptr(), B, H, ci, co,
                                       int(pl), int(relu), self._zero.data_ptr(), st), None, "fac_conv3x3")
            x = y
        return x

    def weighted_features16(self, f: torch.Tensor) -> torch.Tensor:
        """x * GGCA(x) (:436-437) on [B,(1,)7,7,512] 16-bit NHWC."""
        B, (H, W, C) = f.shape[0], f.shape[-3:]
        out = torch.empty_like(f)
        w1, b1, bn4, w2, b2 = self._ggca
        _lib.check(_lib.load().fac_ggca(_lib.DTYPES[self.dtype_name], f.data_ptr(), B, H, W, C, 4, w1.data_ptr(),
                                        b1.data_ptr(), bn4.data_ptr(), w2.data_ptr(), b2.data_ptr(), out.data_ptr(),
                                        torch.cuda.current_stream(f.device).cuda_stream), None, "fac_ggca")
        return out

    def _run(self, src: torch.Tensor, u8: bool, pos_index, want_probs: bool):
        B = src.shape[0]
        dev = src.device
        pidx = _pos_index(B, pos_index, dev)
        f = self.weighted_features16(self.features(src, u8))
        logits = torch.empty(B, SUPPORTED["num_classes"], dtype=torch.float32, device=dev)
        probs = torch.empty_like(logits) if want_probs else None
        _lib.check(_lib.load().fac_forward_features(self._ctx, f.data_ptr(), B, pidx.data_ptr(), None,
                                                    logits.data_ptr(), probs.data_ptr() if want_probs else None,
                                                    torch.cuda.current_stream(dev).cuda_stream), self._ctx,
                   "fac_forward_features")
        return logits, probs

    def forward(self, img: torch.Tensor, mask=None, pos_index=None) -> torch.Tensor:
        poison = mask is not None and reference_mask_poisons(mask, img.shape[0])
        if not img.is_cuda:
            raise RuntimeError("CViT RepBn8 (gfx950 HIP path) needs its input on a GPU device; there is no CPU "
                               "fallback")
        if img.dim() != 4 or tuple(img.shape[1:]) != (3, 224, 224):
            raise ValueError(f"expected img [B,3,224,224], got {tuple(img.shape)}")
        self._prepare(img.device)
        logits = self._run(img.float().contiguous(), False, pos_index, False)[0]
        return logits.fill_(float("nan")) if poison else logits

    def forward_u8(self, crops: torch.Tensor, pos_index=None, return_probs: bool = False):
        """uint8 NHWC RGB crops [B,224,224,3]; x/255 + Normalize fused into the first conv block."""
        if crops.dtype != torch.uint8 or crops.dim() != 4 or tuple(crops.shape[1:]) != (224, 224, 3):
            raise ValueError(f"expected uint8 crops [B,224,224,3], got {crops.dtype} {tuple(crops.shape)}")
        if not crops.is_cuda:
            raise RuntimeError("CViT RepBn8 (gfx950 HIP path) needs its input on a GPU device; there is no CPU "
                               "fallback")
        self._prepare(crops.device)
        logits, probs = self._run(crops.contiguous(), True, pos_index, return_probs)
        return (logits, probs) if return_probs else logits


def _pos_index(B: int, pos_index, device) -> torch.Tensor:
    if pos_index is None:
        if B > MAX_SLOTS:   # `x += self.pos_embedding[0:shape]` (:442-443) raises past 32
            raise RuntimeError(f"The size of tensor a ({B}) must match the size of tensor b ({MAX_SLOTS}) "
                               f"at non-singleton dimension 0")
        return torch.arange(B, dtype=torch.int32, device=device)
    p = torch.as_tensor(pos_index)
    if p.shape != (B,):
        raise ValueError(f"pos_index must have shape ({B},), got {tuple(p.shape)}")
    if p.numel() and not torch.cuda.is_current_stream_capturing() and (int(p.min()) < 0 or int(p.max()) >= MAX_SLOTS):
        raise IndexError(f"pos_index values must lie in [0, {MAX_SLOTS})")
    return p.to(device=device, dtype=torch.int32).contiguous()


__all__ = ["CViT", "TORCH16", "deconv_fold", "sigmoid"]
