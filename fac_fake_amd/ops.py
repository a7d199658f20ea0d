"""Layer-level gfx950 kernels (include/fac_ops.h) on torch device tensors.

The §8f model families (ResVitKan, S3D) are sequences of ordinary layers:
their Python mirrors fold BatchNorm and pack weights once here, then call one
kernel per layer on the current torch stream (capturable into a hipGraph).
Activations are 16-bit channels-last tensors shaped ``[N, D, H, W, C]``
(``D = 1`` for 2-D nets), ``C`` a multiple of 8.  There is no CPU fallback:
every call goes through ``libfac_cvit.so`` and raises if it cannot.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass

import torch

from . import _lib

TORCH16 = {"bf16": torch.bfloat16, "fp16": torch.float16}

RELU, RESID, RELU2, OUT_F32, MAXPOOL3S2, MAXPOOL3S1, PREPOOL3S2 = 1, 2, 4, 8, 16, 32, 64   # FAC_CONV_* flags


class ConvDesc(ctypes.Structure):
    _fields_ = [("dtype", ctypes.c_int), ("inp", ctypes.c_void_p),
                ("n", ctypes.c_int), ("d", ctypes.c_int), ("h", ctypes.c_int), ("w", ctypes.c_int),
                ("cin", ctypes.c_int), ("weight", ctypes.c_void_p), ("bias", ctypes.c_void_p),
                ("cout", ctypes.c_int), ("k_pad", ctypes.c_int),
                ("kd", ctypes.c_int), ("kh", ctypes.c_int), ("kw", ctypes.c_int),
                ("sd", ctypes.c_int), ("sh", ctypes.c_int), ("sw", ctypes.c_int),
                ("pd", ctypes.c_int), ("ph", ctypes.c_int), ("pw", ctypes.c_int),
                ("od", ctypes.c_int), ("oh", ctypes.c_int), ("ow", ctypes.c_int),
                ("out", ctypes.c_void_p), ("ldo", ctypes.c_int), ("c_off", ctypes.c_int),
                ("residual", ctypes.c_void_p), ("ldr", ctypes.c_int), ("r_off", ctypes.c_int),
                ("flags", ctypes.c_int)]


class PoolDesc(ctypes.Structure):
    _fields_ = [("dtype", ctypes.c_int), ("inp", ctypes.c_void_p),
                ("n", ctypes.c_int), ("d", ctypes.c_int), ("h", ctypes.c_int), ("w", ctypes.c_int),
                ("c", ctypes.c_int),
                ("kd", ctypes.c_int), ("kh", ctypes.c_int), ("kw", ctypes.c_int),
                ("sd", ctypes.c_int), ("sh", ctypes.c_int), ("sw", ctypes.c_int),
                ("pd", ctypes.c_int), ("ph", ctypes.c_int), ("pw", ctypes.c_int),
                ("od", ctypes.c_int), ("oh", ctypes.c_int), ("ow", ctypes.c_int),
                ("mode", ctypes.c_int), ("out", ctypes.c_void_p), ("ldo", ctypes.c_int), ("c_off", ctypes.c_int)]


_ZERO256: dict = {}


def _zero256(device: torch.device) -> torch.Tensor:
    """256 zero bytes of device memory: the source of conv.hip's zero-padding loads."""
    key = (device.type, device.index)
    if key not in _ZERO256:
        if torch.cuda.is_current_stream_capturing():
            raise RuntimeError("the zero page must be allocated before graph capture (construct the layers first)")
        _ZERO256[key] = torch.zeros(128, dtype=torch.int16, device=device)
    return _ZERO256[key]


def _stream(t: torch.Tensor):
    return torch.cuda.current_stream(t.device).cuda_stream


def _triple(v):
    if isinstance(v, int):
        return (v, v, v)
    v = tuple(v)
    return (1,) * (3 - len(v)) + v if len(v) < 3 else v


def _pads(v):
    if isinstance(v, int):
        return (v, v, v)
    v = tuple(v)
    return (0,) * (3 - len(v)) + v if len(v) < 3 else v


def fold_bn(weight: torch.Tensor, bias, gamma, beta, mean, var, eps: float):
    """Eval-mode BatchNorm folded into the preceding conv, in fp32 on the host:
    s = gamma / sqrt(var + eps), W' = W s, b' = (b - mean) s + beta."""
    w = weight.detach().to("cpu", torch.float32)
    co = w.shape[0]
    b = bias.detach().to("cpu", torch.float32) if bias is not None else torch.zeros(co)
    if gamma is None:
        return w, b
    s = gamma.detach().float().cpu() / torch.sqrt(var.detach().float().cpu() + eps)
    w = w * s.view(-1, *([1] * (w.dim() - 1)))
    b = (b - mean.detach().float().cpu()) * s + beta.detach().float().cpu()
    return w, b


@dataclass
class ConvGeom:
    kd: int
    kh: int
    kw: int
    sd: int
    sh: int
    sw: int
    pd: int
    ph: int
    pw: int


class ConvLayer:
    """A conv (+ folded BN) packed for fac_conv_nd: weights 16-bit
    [cout_pad][k_pad] with k = ((tz*kh + ty)*kw + tx)*cin_p + c."""

    def __init__(self, weight: torch.Tensor, bias: torch.Tensor, stride=1, padding=0, *, dtype: str, device,
                 cin_pad: int | None = None):
        w = weight.detach().to("cpu", torch.float32)
        if w.dim() == 4:                             # Conv2d: [co, ci, kh, kw] -> depth 1, no depth stride/pad
            w = w.unsqueeze(2)
            st = (1,) + ((stride, stride) if isinstance(stride, int) else tuple(stride))
            pd = (0,) + ((padding, padding) if isinstance(padding, int) else tuple(padding))
        else:
            st, pd = _triple(stride), _pads(padding)
        co, ci, kd, kh, kw = w.shape
        self.cout, self.cin = co, ci
        self.cin_p = cin_pad or (ci + 7) // 8 * 8
        self.g = ConvGeom(kd, kh, kw, *st, *pd)
        lib = _lib.load()
        cp, kp = ctypes.c_int(), ctypes.c_int()
        _lib.check(lib.fac_conv_weight_layout(co, self.cin_p, kd, kh, kw, ctypes.byref(cp), ctypes.byref(kp)), None,
                   "fac_conv_weight_layout")
        self.cout_pad, self.k_pad = cp.value, kp.value
        wp = torch.zeros(co, kd, kh, kw, self.cin_p)
        wp[..., :ci] = w.permute(0, 2, 3, 4, 1)
        packed = torch.zeros(self.cout_pad, self.k_pad)
        packed[:co, :kd * kh * kw * self.cin_p] = wp.reshape(co, -1)
        self.dtype = dtype
        self.w = packed.to(TORCH16[dtype]).to(device)
        b = torch.zeros(self.cout_pad)
        b[:co] = bias.detach().to("cpu", torch.float32)
        self.b = b.to(device)
        # 3x3 / stride 1 / padding 1 spatial convs with 32-channel chunks (the
        # ResNet-50 and S3D (1,3,3) layers) run on the CViT conv-stack kernel
        # (conv.hip: halo staged once per 32-channel chunk for all 9 taps)
        # wherever it has a tile for the resolution and width: packed per
        # input size on first use (fac_conv3x3_pack), else fac_conv_nd.
        self._w33 = None
        g = self.g
        if (kd, kh, kw) == (1, 3, 3) and (g.sd, g.sh, g.sw) == (1, 1, 1) and (g.pd, g.ph, g.pw) == (0, 1, 1) \
                and ci % 32 == 0:
            self._w33 = w[:, :, 0].reshape(co, ci, 9).contiguous()
            self._pk33 = {}
            self._device = device
            _zero256(torch.device(device))  # allocated (and zeroed) before any graph capture
            # conv.hip weights are packed on first use per input size (a
            # synchronous host->device copy: run one eager forward before
            # graph capture, which every caller here does), so a layer holds
            # only the packings of the sizes it sees

    def _packed33(self, h: int):
        """fac_conv3x3 weights for h x h inputs, or None if conv.hip has no tile for it."""
        if h not in self._pk33:
            if torch.cuda.is_current_stream_capturing():
                # packing copies host -> device synchronously: illegal inside a capture
                raise RuntimeError(f"conv weights for {h}x{h} inputs are packed on first use: run one eager "
                                   "forward (or the model's reserve()) at this input size before graph capture")
            lib = _lib.load()
            n = lib.fac_conv3x3_packed_elems(h, self.cin, self.cout)
            pk = None
            if n:
                out = torch.empty(n, dtype=torch.int16)
                _lib.check(lib.fac_conv3x3_pack(_lib.DTYPES[self.dtype], h, self.cin, self.cout, self._w33.data_ptr(),
                                                out.data_ptr()), None, "fac_conv3x3_pack")
                pk = out.view(TORCH16[self.dtype]).to(self._device)
            self._pk33[h] = pk
        return self._pk33[h]

    # maps the S3D drop-in fuses branch3's pool on: the kernel also takes 3 x 3,
    # where the chain of 13 dependent 64-channel chunks per unit measured
    # slower than the pool + conv launches (94 vs ~59 us at 1536 clips)
    MAXPOOL3S1_MAPS = (14, 7)

    def maxpool3s1_ok(self, x: torch.Tensor, out: torch.Tensor | None = None, c_off: int = 0) -> bool:
        """Whether fac_conv_nd takes FAC_CONV_MAXPOOL3S1 for this layer on x
        (ops.hip maxpool3_pw)."""
        g = self.g
        _, _, h, w, _ = x.shape
        return ((g.kd, g.kh, g.kw, g.sd, g.sh, g.sw, g.pd, g.ph, g.pw) == (1, 1, 1, 1, 1, 1, 0, 0, 0)
                and h == w and h in self.MAXPOOL3S1_MAPS and self.cout % 32 == 0 and c_off % 8 == 0
                and (out is None or out.shape[4] % 8 == 0) and _lib.exports("fac_conv_nd"))

    def prepool3s2_ok(self, x: torch.Tensor) -> bool:
        """Whether fac_conv_nd takes FAC_CONV_PREPOOL3S2 for this layer on x:
        MaxPool3d((1,3,3), (1,2,2), (0,1,1)) of x, then this 1x1x1 64 -> 64
        conv (S3D's base.1 + base.2 at 112^2 clips, ops.hip maxpool2s_pw)."""
        g = self.g
        return ((g.kd, g.kh, g.kw, g.sd, g.sh, g.sw, g.pd, g.ph, g.pw) == (1, 1, 1, 1, 1, 1, 0, 0, 0)
                and self.cin == 64 and self.cin_p == 64 and self.cout == 64 and x.shape[3] == 56
                and x.shape[4] == 64)

    def out_dims(self, d, h, w):
        g = self.g
        return ((d + 2 * g.pd - g.kd) // g.sd + 1, (h + 2 * g.ph - g.kh) // g.sh + 1,
                (w + 2 * g.pw - g.kw) // g.sw + 1)

    def __call__(self, x: torch.Tensor, *, relu: bool = True, out: torch.Tensor | None = None, c_off: int = 0,
                 residual: torch.Tensor | None = None, relu2: bool = False, out_f32: bool = False,
                 maxpool3s2: bool = False, maxpool3s1: bool = False, prepool3s2: bool = False) -> torch.Tensor:
        """maxpool3s2: MaxPool2d(3, 2, 1) over H, W fused into the launch
        (FAC_CONV_MAXPOOL3S2: the space-to-depth first conv with relu only;
        the output is the pooled [N, D, Ho/2, Wo/2, C]).  maxpool3s1:
        MaxPool3d(3, 1, 1) over the INPUT first (FAC_CONV_MAXPOOL3S1: a 1x1x1
        conv on a 14 / 7 / 3 square map, cout % 32 == 0; maxpool3s1_ok).
        prepool3s2: MaxPool3d((1,3,3), (1,2,2), (0,1,1)) over the INPUT
        first, the output at the pooled positions (FAC_CONV_PREPOOL3S2:
        prepool3s2_ok)."""
        n, d, h, w, c = x.shape
        if c != self.cin_p or x.dtype != TORCH16[self.dtype] or not x.is_contiguous():
            raise ValueError(f"conv input must be contiguous {self.dtype} [N,D,H,W,{self.cin_p}], got "
                             f"{x.dtype} {tuple(x.shape)}")
        od, oh, ow = self.out_dims(d, h, w)
        if prepool3s2:
            if not self.prepool3s2_ok(x) or residual is not None or relu2 or out_f32 or maxpool3s2 or maxpool3s1:
                raise ValueError("prepool3s2 needs a 1x1x1 64 -> 64 conv on a 56-wide map, no residual / relu2 / "
                                 "fp32 output / other pool")
            oh, ow = (h - 1) // 2 + 1, (w - 1) // 2 + 1
        if maxpool3s2:
            if not relu or residual is not None or relu2 or out_f32 or c_off or oh % 2 or ow % 2:
                raise ValueError("maxpool3s2 needs relu, no residual / relu2 / fp32 output, even output dims")
            oh, ow = oh // 2, ow // 2
        if out is None:
            out = torch.empty(n, od, oh, ow, self.cout, device=x.device,
                              dtype=torch.float32 if out_f32 else x.dtype)
        if tuple(out.shape[:4]) != (n, od, oh, ow) or not out.is_contiguous():
            raise ValueError(f"conv output must be contiguous [{n},{od},{oh},{ow},C], got {tuple(out.shape)}")
        if maxpool3s1 and (not self.maxpool3s1_ok(x, out, c_off) or residual is not None or relu2 or out_f32):
            raise ValueError("maxpool3s1 needs a 1x1x1 conv over a 14 / 7 / 3 square map, cout % 32 == 0, "
                             "no residual / relu2 / fp32 output, ldo and c_off % 8 == 0")
        if (self._w33 is not None and h == w and residual is None and not relu2 and not out_f32 and c_off == 0
                and not maxpool3s2 and not maxpool3s1 and not prepool3s2 and out.shape[4] == self.cout and self.cin_p == self.cin):
            pk = self._packed33(h)
            if pk is not None:
                lib = _lib.load()
                _lib.check(lib.fac_conv3x3(_lib.DTYPES[self.dtype], x.data_ptr(), pk.data_ptr(), self.b.data_ptr(),
                                           out.data_ptr(), n * d, h, self.cin, self.cout, 0, 1 if relu else 0,
                                           _zero256(x.device).data_ptr(), _stream(x)), None, "fac_conv3x3")
                return out
        g = self.g
        dsc = ConvDesc()
        dsc.dtype = _lib.DTYPES[self.dtype]
        dsc.inp = x.data_ptr()
        dsc.n, dsc.d, dsc.h, dsc.w, dsc.cin = n, d, h, w, c
        dsc.weight, dsc.bias = self.w.data_ptr(), self.b.data_ptr()
        dsc.cout, dsc.k_pad = self.cout, self.k_pad
        dsc.kd, dsc.kh, dsc.kw, dsc.sd, dsc.sh, dsc.sw = g.kd, g.kh, g.kw, g.sd, g.sh, g.sw
        dsc.pd, dsc.ph, dsc.pw = g.pd, g.ph, g.pw
        dsc.od, dsc.oh, dsc.ow = (od, 2 * oh, 2 * ow) if maxpool3s2 else (od, oh, ow)
        dsc.out, dsc.ldo, dsc.c_off = out.data_ptr(), out.shape[4], c_off
        flags = (RELU if relu else 0) | (RELU2 if relu2 else 0) | (OUT_F32 if out_f32 else 0) | \
            (MAXPOOL3S2 if maxpool3s2 else 0) | (MAXPOOL3S1 if maxpool3s1 else 0) | \
            (PREPOOL3S2 if prepool3s2 else 0)
        if residual is not None:
            if tuple(residual.shape[:4]) != (n, od, oh, ow) or residual.dtype != x.dtype:
                raise ValueError("residual must match the output positions and dtype")
            dsc.residual, dsc.ldr, dsc.r_off = residual.data_ptr(), residual.shape[4], 0
            flags |= RESID
        dsc.flags = flags
        _lib.check(_lib.load().fac_conv_nd(ctypes.byref(dsc), _stream(x)), None, "fac_conv_nd")
        return out


def _desc(layer: ConvLayer, x: torch.Tensor, out: torch.Tensor | None, flags: int) -> "ConvDesc":
    n, d, h, w, c = x.shape
    if c != layer.cin_p or x.dtype != TORCH16[layer.dtype] or not x.is_contiguous():
        raise ValueError(f"conv input must be contiguous {layer.dtype} [N,D,H,W,{layer.cin_p}], got "
                         f"{x.dtype} {tuple(x.shape)}")
    od, oh, ow = layer.out_dims(d, h, w)
    g = layer.g
    dsc = ConvDesc()
    dsc.dtype = _lib.DTYPES[layer.dtype]
    dsc.inp = x.data_ptr()
    dsc.n, dsc.d, dsc.h, dsc.w, dsc.cin = n, d, h, w, c
    dsc.weight, dsc.bias = layer.w.data_ptr(), layer.b.data_ptr()
    dsc.cout, dsc.k_pad = layer.cout, layer.k_pad
    dsc.kd, dsc.kh, dsc.kw, dsc.sd, dsc.sh, dsc.sw = g.kd, g.kh, g.kw, g.sd, g.sh, g.sw
    dsc.pd, dsc.ph, dsc.pw = g.pd, g.ph, g.pw
    dsc.od, dsc.oh, dsc.ow = od, oh, ow
    if out is not None:
        dsc.out, dsc.ldo, dsc.c_off = out.data_ptr(), out.shape[4], 0
    dsc.flags = flags
    return dsc


def conv_dual(layer: ConvLayer, h: torch.Tensor, ds: ConvLayer, x: torch.Tensor,
              out: torch.Tensor | None = None) -> torch.Tensor:
    """relu(relu(layer(h)) + ds(x)) in one fac_conv_nd_dual launch: a ResNet
    bottleneck's conv3 + bn3 + ReLU with its downsample branch (conv + bn,
    ResVitKan.py:146-152) added before the final ReLU, without the
    downsample output going through memory.  Same result as
    ``layer(h, residual=ds(x, relu=False), relu2=True)`` up to fp32 rounding
    (the downsample's sum is not rounded to 16 bits first)."""
    n, d, hh, w, _ = h.shape
    od, oh, ow = layer.out_dims(d, hh, w)
    if tuple(ds.out_dims(*x.shape[1:4])) != (od, oh, ow) or x.shape[0] != n or ds.cout != layer.cout:
        raise ValueError("conv_dual: the two convs must produce the same output positions and channels")
    if out is None:
        out = torch.empty(n, od, oh, ow, layer.cout, device=h.device, dtype=h.dtype)
    d1 = _desc(layer, h, out, RELU | RELU2)
    d2 = _desc(ds, x, None, 0)
    _lib.check(_lib.load().fac_conv_nd_dual(ctypes.byref(d1), ctypes.byref(d2), _stream(h)), None,
               "fac_conv_nd_dual")
    return out


def bottleneck_pw2(c3: ConvLayer, h: torch.Tensor, res: torch.Tensor, c1: ConvLayer):
    """(x, h1) = (relu(relu(c3(h)) + res), c1(x)) in one fac_bottleneck_pw2
    launch: a ResNet-50 layer1 bottleneck's conv3 (+ bn3, identity residual)
    and the next block's conv1 (+ bn1 + ReLU), the 256-channel block output
    written once and not read back (ResVitKan.py:146-152).  Same values as
    ``c3(h, residual=res, relu2=True)`` then ``c1(x)`` up to fp32 summation
    order."""
    n, d, hh, w, _ = h.shape
    x = torch.empty(n, d, hh, w, c3.cout, device=h.device, dtype=h.dtype)
    h1 = torch.empty(n, d, hh, w, c1.cout, device=h.device, dtype=h.dtype)
    if tuple(res.shape) != tuple(x.shape) or res.dtype != h.dtype or not res.is_contiguous():
        raise ValueError("bottleneck_pw2: residual must be the block input [N,D,H,W,256]")
    d3 = _desc(c3, h, x, RELU | RESID | RELU2)
    d3.residual, d3.ldr, d3.r_off = res.data_ptr(), res.shape[4], 0
    d1 = _desc(c1, x, h1, RELU)
    _lib.check(_lib.load().fac_bottleneck_pw2(ctypes.byref(d3), ctypes.byref(d1), _stream(h)), None,
               "fac_bottleneck_pw2")
    return x, h1


def conv_split(layer: ConvLayer, x: torch.Tensor, splits, out0: torch.Tensor, c_off0: int, out1: torch.Tensor,
               out2: torch.Tensor, relu: bool = True) -> None:
    """One fac_conv_nd_split launch of `layer` (a conv over concatenated
    output channels): columns [0, s1) -> out0[..., c_off0:], [s1, s2) -> out1,
    [s2, cout) -> out2 (each [N,D,H,W,C] contiguous)."""
    s1, s2 = splits
    n, d, h, w, c = x.shape
    if c != layer.cin_p or x.dtype != TORCH16[layer.dtype] or not x.is_contiguous():
        raise ValueError("conv_split input must be a contiguous 16-bit [N,D,H,W,cin] tensor")
    od, oh, ow = layer.out_dims(d, h, w)
    for t, width in ((out1, s2 - s1), (out2, layer.cout - s2)):
        if tuple(t.shape[:4]) != (n, od, oh, ow) or t.shape[4] < width or not t.is_contiguous():
            raise ValueError("conv_split outputs must be contiguous [N,D,H,W,C] tensors wide enough")
    g = layer.g
    dsc = ConvDesc()
    dsc.dtype = _lib.DTYPES[layer.dtype]
    dsc.inp = x.data_ptr()
    dsc.n, dsc.d, dsc.h, dsc.w, dsc.cin = n, d, h, w, c
    dsc.weight, dsc.bias = layer.w.data_ptr(), layer.b.data_ptr()
    dsc.cout, dsc.k_pad = layer.cout, layer.k_pad
    dsc.kd, dsc.kh, dsc.kw, dsc.sd, dsc.sh, dsc.sw = g.kd, g.kh, g.kw, g.sd, g.sh, g.sw
    dsc.pd, dsc.ph, dsc.pw = g.pd, g.ph, g.pw
    dsc.od, dsc.oh, dsc.ow = od, oh, ow
    dsc.out, dsc.ldo, dsc.c_off = out0.data_ptr(), out0.shape[4], c_off0
    dsc.flags = RELU if relu else 0
    _lib.check(_lib.load().fac_conv_nd_split(ctypes.byref(dsc), out1.data_ptr(), out1.shape[4], s1, out2.data_ptr(),
                                             out2.shape[4], s2, _stream(x)), None, "fac_conv_nd_split")


def pool(x: torch.Tensor, kernel, stride, padding=0, mode: str = "max", out: torch.Tensor | None = None,
         c_off: int = 0) -> torch.Tensor:
    n, d, h, w, c = x.shape
    (kd, kh, kw), (sd, sh, sw), (pd, ph, pw) = _triple(kernel), _triple(stride), _pads(padding)
    od, oh, ow = (d + 2 * pd - kd) // sd + 1, (h + 2 * ph - kh) // sh + 1, (w + 2 * pw - kw) // sw + 1
    if out is None:
        out = torch.empty(n, od, oh, ow, c, device=x.device, dtype=x.dtype)
    dsc = PoolDesc()
    dsc.dtype = 0 if x.dtype == torch.bfloat16 else 1
    dsc.inp = x.data_ptr()
    dsc.n, dsc.d, dsc.h, dsc.w, dsc.c = n, d, h, w, c
    dsc.kd, dsc.kh, dsc.kw, dsc.sd, dsc.sh, dsc.sw, dsc.pd, dsc.ph, dsc.pw = kd, kh, kw, sd, sh, sw, pd, ph, pw
    dsc.od, dsc.oh, dsc.ow = od, oh, ow
    dsc.mode = {"max": 0, "avg": 1}[mode]
    dsc.out, dsc.ldo, dsc.c_off = out.data_ptr(), out.shape[4], c_off
    _lib.check(_lib.load().fac_pool_nd(ctypes.byref(dsc), _stream(x)), None, "fac_pool_nd")
    return out


def max_pool_sep(x: torch.Tensor, kernel, stride, padding=0) -> torch.Tensor:
    """Max pooling.  MaxPool3d(3, 1, 1) and strided windows are one
    fac_pool_nd call (a sliding-window kernel / a direct pass: for S3D's
    (1,3,3)/(1,2,2), (3,3,3)/2, (2,2,2)/2 and ResNet's 3x3/2 one direct pass
    over the 4-8x smaller output beat the separable passes, same-box S3D
    29.4k -> 30.35k clips/s); other stride-1 windows are one fac_pool_nd pass
    per axis (W, then H, then D; axes with kernel 1, stride 1 and no padding
    are skipped).  A max over a box window (padding ignored, i.e. -inf) is
    the max over its rows of the max over its columns, so every form is
    bit-identical to one 3-D pass."""
    k, s, p = _triple(kernel), _triple(stride), _pads(padding)
    if (k == (3, 3, 3) and s == (1, 1, 1) and p == (1, 1, 1)) or s != (1, 1, 1):
        return pool(x, kernel, stride, padding, "max")
    y = x
    for ax in (2, 1, 0):
        if k[ax] == 1 and s[ax] == 1 and p[ax] == 0:
            continue
        kk, ss, pp = [1, 1, 1], [1, 1, 1], [0, 0, 0]
        kk[ax], ss[ax], pp[ax] = k[ax], s[ax], p[ax]
        y = pool(y, tuple(kk), tuple(ss), tuple(pp), "max")
    return y if y is not x else pool(x, kernel, stride, padding, "max")


def pack_input(src: torch.Tensor, *, dtype: str, u8: bool, div: float = 1.0, mean=None, std=None,
               spatial: tuple[int, ...]) -> torch.Tensor:
    """3-channel images -> 16-bit [N, D, H, W, 8] (fac_pack_input).
    u8: src uint8 [N, *spatial, 3]; else fp32 planar [N, 3, *spatial]."""
    n = src.shape[0]
    s = 1
    for v in spatial:
        s *= v
    d, h, w = (1,) * (3 - len(spatial)) + tuple(spatial)
    out = torch.empty(n, d, h, w, 8, device=src.device, dtype=TORCH16[dtype])
    m = (ctypes.c_float * 3)(*(mean if mean is not None else (0.0, 0.0, 0.0)))
    sd = (ctypes.c_float * 3)(*(std if std is not None else (1.0, 1.0, 1.0)))
    src = src.contiguous()
    _lib.check(_lib.load().fac_pack_input(_lib.DTYPES[dtype], src.data_ptr(), 0 if u8 else 1, n, s, float(div),
                                          ctypes.cast(m, ctypes.c_void_p), ctypes.cast(sd, ctypes.c_void_p),
                                          out.data_ptr(), 8, _stream(src)), None, "fac_pack_input")
    return out


def pack_input_s2d(src: torch.Tensor, *, dtype: str, u8: bool, div: float = 1.0, mean=None, std=None,
                   pad_before: int = 2, pad_after: int = 1) -> torch.Tensor:
    """3-channel images -> 16-bit space-to-depth cells [N, T, h/2+pb+pa, w/2+pb+pa, 16]
    (fac_pack_input_s2d).  u8: src uint8 [N, h, w, 3] (T = 1); else fp32
    [N, 3, h, w] (T = 1) or a clip batch [N, 3, T, h, w]."""
    n = src.shape[0]
    frames = src.shape[2] if (not u8 and src.dim() == 5) else 1
    h, w = (src.shape[1], src.shape[2]) if u8 else (src.shape[-2], src.shape[-1])
    ho, wo = h // 2 + pad_before + pad_after, w // 2 + pad_before + pad_after
    out = torch.empty(n, frames, ho, wo, 16, device=src.device, dtype=TORCH16[dtype])
    m = (ctypes.c_float * 3)(*(mean if mean is not None else (0.0, 0.0, 0.0)))
    sd = (ctypes.c_float * 3)(*(std if std is not None else (1.0, 1.0, 1.0)))
    src = src.contiguous()
    _lib.check(_lib.load().fac_pack_input_s2d(_lib.DTYPES[dtype], src.data_ptr(), 0 if u8 else 1, n, frames, h, w,
                                              pad_before, pad_after, float(div), ctypes.cast(m, ctypes.c_void_p),
                                              ctypes.cast(sd, ctypes.c_void_p), out.data_ptr(), _stream(src)),
               None, "fac_pack_input_s2d")
    return out


def conv_s2d4_clip(layer: ConvLayer, clip: torch.Tensor, *, pad_before: int = 2, pad_after: int = 1,
                   relu: bool = True) -> torch.Tensor:
    """``layer(pack_input_s2d(clip, u8=False, pad_before, pad_after))`` in one
    launch (fac_conv_s2d4_clip): S3D's base.0 spatial (1,7,7)/(1,2,2) conv
    (model.py:18) with the space-to-depth packing folded into the conv's halo
    staging, so the 16-bit cell image never goes through HBM.  ``clip`` is the
    fp32 batch [N, 3, T, h, w], or uint8 (fac_conv_s2d4_clip_u8: decoded
    frames, a quarter of the bytes, the output of the same clip cast to fp32);
    ``layer`` the s2d-weight 4x4 conv.  Bit-identical to the two launches."""
    if clip.dtype not in (torch.float32, torch.uint8) or clip.dim() != 5 or clip.shape[1] != 3 or \
            not clip.is_contiguous():
        raise ValueError(f"expected a contiguous fp32 / uint8 clip [N,3,T,H,W], got {clip.dtype} {tuple(clip.shape)}")
    n, _, t, h, w = clip.shape
    hc, wc = h // 2 + pad_before + pad_after, w // 2 + pad_before + pad_after
    od, oh, ow = layer.out_dims(t, hc, wc)
    out = torch.empty(n, od, oh, ow, layer.cout, device=clip.device, dtype=TORCH16[layer.dtype])
    g = layer.g
    dsc = ConvDesc()
    dsc.dtype = _lib.DTYPES[layer.dtype]
    dsc.n, dsc.d, dsc.h, dsc.w, dsc.cin = n, t, hc, wc, layer.cin_p
    dsc.weight, dsc.bias = layer.w.data_ptr(), layer.b.data_ptr()
    dsc.cout, dsc.k_pad = layer.cout, layer.k_pad
    dsc.kd, dsc.kh, dsc.kw, dsc.sd, dsc.sh, dsc.sw = g.kd, g.kh, g.kw, g.sd, g.sh, g.sw
    dsc.pd, dsc.ph, dsc.pw = g.pd, g.ph, g.pw
    dsc.od, dsc.oh, dsc.ow = od, oh, ow
    dsc.out, dsc.ldo, dsc.c_off = out.data_ptr(), layer.cout, 0
    dsc.flags = RELU if relu else 0
    fn = "fac_conv_s2d4_clip_u8" if clip.dtype == torch.uint8 else "fac_conv_s2d4_clip"
    _lib.check(getattr(_lib.load(), fn)(ctypes.byref(dsc), clip.data_ptr(), h, w, pad_before, _stream(clip)), None, fn)
    return out


def sep_mid_ok(spatial: ConvLayer, temporal: ConvLayer, x: torch.Tensor) -> bool:
    """Whether fac_sep_mid takes this SepConv3d on x: Mixed_3c's branch2
    (1,3,3) 32 -> 96 (output rows zero-padded to 128) then (3,1,1) 128 -> 96
    over [N, 8, 14, 14, 32]."""
    gs, gt = spatial.g, temporal.g
    return (x.dim() == 5 and tuple(x.shape[1:]) == (8, 14, 14, 32) and spatial.cin_p == 32 and spatial.cout == 128
            and (gs.kd, gs.kh, gs.kw, gs.sd, gs.sh, gs.sw, gs.pd, gs.ph, gs.pw) == (1, 3, 3, 1, 1, 1, 0, 1, 1)
            and temporal.cin_p == 128 and temporal.cout == 96
            and (gt.kd, gt.kh, gt.kw, gt.sd, gt.sh, gt.sw, gt.pd, gt.ph, gt.pw) == (3, 1, 1, 1, 1, 1, 1, 0, 0)
            and _lib.exports("fac_sep_mid"))


def sep_tiny_ok(spatial: ConvLayer, temporal: ConvLayer, x: torch.Tensor) -> bool:
    """Whether fac_sep_tiny takes this SepConv3d on x: Mixed_3b's branch2
    (1,3,3) 16 -> 32 then (3,1,1) 32 -> 32 over [N, 8, 14, 14, 16]."""
    gs, gt = spatial.g, temporal.g
    return (x.dim() == 5 and tuple(x.shape[1:]) == (8, 14, 14, 16) and spatial.cin_p == 16 and spatial.cout == 32
            and (gs.kd, gs.kh, gs.kw, gs.sd, gs.sh, gs.sw, gs.pd, gs.ph, gs.pw) == (1, 3, 3, 1, 1, 1, 0, 1, 1)
            and temporal.cin_p == 32 and temporal.cout == 32
            and (gt.kd, gt.kh, gt.kw, gt.sd, gt.sh, gt.sw, gt.pd, gt.ph, gt.pw) == (3, 1, 1, 1, 1, 1, 1, 0, 0)
            and _lib.exports("fac_sep_tiny"))


def sep_tiny(spatial: ConvLayer, temporal: ConvLayer, x: torch.Tensor, out: torch.Tensor, c_off: int = 0) -> torch.Tensor:
    """``temporal(spatial(x))`` with both ReLUs in one launch, written into
    channels [c_off, c_off + cout) of `out` [N, 8, 14, 14, C]: fac_sep_tiny
    (Mixed_3b's branch2 SepConv, the 32-channel map kept in LDS) or, for
    Mixed_3c's 32 -> 96 -> 96 one, fac_sep_mid (2-row bands, the 96-channel
    map in LDS)."""
    mid = sep_mid_ok(spatial, temporal, x)
    if not (mid or sep_tiny_ok(spatial, temporal, x)) or x.dtype != TORCH16[spatial.dtype] or not x.is_contiguous():
        raise ValueError(f"sep_tiny needs Mixed_3b's / 3c's branch2 SepConv over [N,8,14,14,16|32], got "
                         f"{tuple(x.shape)}")
    if tuple(out.shape[:4]) != tuple(x.shape[:4]) or not out.is_contiguous():
        raise ValueError("out must be contiguous [N,8,14,14,C]")
    sd = _desc(spatial, x, None, RELU)
    n = x.shape[0]
    td = ConvDesc()
    td.dtype = _lib.DTYPES[temporal.dtype]
    td.n, td.d, td.h, td.w, td.cin = n, 8, 14, 14, temporal.cin_p
    td.weight, td.bias = temporal.w.data_ptr(), temporal.b.data_ptr()
    td.cout, td.k_pad = temporal.cout, temporal.k_pad
    g = temporal.g
    td.kd, td.kh, td.kw, td.sd, td.sh, td.sw = g.kd, g.kh, g.kw, g.sd, g.sh, g.sw
    td.pd, td.ph, td.pw = g.pd, g.ph, g.pw
    td.od, td.oh, td.ow = temporal.out_dims(8, 14, 14)
    td.out, td.ldo, td.c_off = out.data_ptr(), out.shape[4], c_off
    td.flags = RELU
    fn = "fac_sep_mid" if mid else "fac_sep_tiny"
    _lib.check(getattr(_lib.load(), fn)(ctypes.byref(sd), ctypes.byref(td), _stream(x)), None, fn)
    return out


def s3d_base0_u8(spatial: ConvLayer, temporal: ConvLayer, clip: torch.Tensor, *, pad_before: int = 2,
                 pad_after: int = 1) -> torch.Tensor:
    """S3D's base.0 in one launch (fac_s3d_base0_u8): ``temporal(
    conv_s2d4_clip(spatial, clip))`` for a uint8 clip batch [N, 3, 16, 112,
    112], both halves + ReLU, without the 16-frame half-resolution map going
    through HBM; bit-identical to the two launches.  -> [N, 8, 56, 56, 64]."""
    if clip.dtype != torch.uint8 or clip.dim() != 5 or clip.shape[1] != 3 or not clip.is_contiguous():
        raise ValueError(f"expected a contiguous uint8 clip [N,3,16,H,W], got {clip.dtype} {tuple(clip.shape)}")
    n, _, t, h, w = clip.shape
    hc, wc = h // 2 + pad_before + pad_after, w // 2 + pad_before + pad_after
    od, oh, ow = spatial.out_dims(t, hc, wc)
    g = spatial.g
    sd = ConvDesc()
    sd.dtype = _lib.DTYPES[spatial.dtype]
    sd.n, sd.d, sd.h, sd.w, sd.cin = n, t, hc, wc, spatial.cin_p
    sd.weight, sd.bias = spatial.w.data_ptr(), spatial.b.data_ptr()
    sd.cout, sd.k_pad = spatial.cout, spatial.k_pad
    sd.kd, sd.kh, sd.kw, sd.sd, sd.sh, sd.sw = g.kd, g.kh, g.kw, g.sd, g.sh, g.sw
    sd.pd, sd.ph, sd.pw = g.pd, g.ph, g.pw
    sd.od, sd.oh, sd.ow = od, oh, ow
    sd.ldo, sd.flags = spatial.cout, RELU
    tod, toh, tow = temporal.out_dims(od, oh, ow)
    out = torch.empty(n, tod, toh, tow, temporal.cout, device=clip.device, dtype=TORCH16[temporal.dtype])
    tg = temporal.g
    td = ConvDesc()
    td.dtype = _lib.DTYPES[temporal.dtype]
    td.n, td.d, td.h, td.w, td.cin = n, od, oh, ow, temporal.cin_p
    td.weight, td.bias = temporal.w.data_ptr(), temporal.b.data_ptr()
    td.cout, td.k_pad = temporal.cout, temporal.k_pad
    td.kd, td.kh, td.kw, td.sd, td.sh, td.sw = tg.kd, tg.kh, tg.kw, tg.sd, tg.sh, tg.sw
    td.pd, td.ph, td.pw = tg.pd, tg.ph, tg.pw
    td.od, td.oh, td.ow = tod, toh, tow
    td.out, td.ldo, td.c_off = out.data_ptr(), temporal.cout, 0
    td.flags = RELU
    _lib.check(_lib.load().fac_s3d_base0_u8(ctypes.byref(sd), ctypes.byref(td), clip.data_ptr(), h, w, pad_before,
                                            _stream(clip)), None, "fac_s3d_base0_u8")
    return out


def s2d_weight(w: torch.Tensor) -> torch.Tensor:
    """[co, 3, 7, 7] stride-2 pad-3 kernel -> [co, 16, 4, 4] stride-1 kernel over
    fac_pack_input_s2d cells: w'[o][(dy*2+dx)*4 + c][ty][tx] = w[o][c][2ty+dy-1][2tx+dx-1].
    A (1, 7, 7) Conv3d kernel maps to (1, 4, 4) the same way."""
    if w.dim() == 5:
        if w.shape[2] != 1:
            raise ValueError("space-to-depth packing is for spatial-only (1, k, k) kernels")
        return s2d_weight(w[:, :, 0]).unsqueeze(2)
    co, ci, kh, kw = w.shape
    if ci != 3 or kh != 7 or kw != 7:
        raise ValueError("space-to-depth packing is for the 3-channel 7x7/2 first conv")
    out = torch.zeros(co, 16, 4, 4, dtype=w.dtype)
    for ty in range(4):
        for dy in range(2):
            ky = 2 * ty + dy - 1
            if not 0 <= ky < 7:
                continue
            for tx in range(4):
                for dx in range(2):
                    kx = 2 * tx + dx - 1
                    if 0 <= kx < 7:
                        out[:, (dy * 2 + dx) * 4:(dy * 2 + dx) * 4 + 3, ty, tx] = w[:, :, ky, kx]
    return out


class KANLinearLayer:
    """KANLinear (CViT-main/ResVitKan/kan.py:18-206) packed for fac_kan_linear:
    wcat[i][0][o] = base_weight[o][i], wcat[i][1+k][o] = spline_weight[o][i][k] * spline_scaler[o][i]."""

    N_KNOTS = 12

    def __init__(self, grid, base_weight, spline_weight, spline_scaler, device):
        g = grid.detach().to("cpu", torch.float32)
        bw = base_weight.detach().to("cpu", torch.float32)
        sw = spline_weight.detach().to("cpu", torch.float32)
        ss = spline_scaler.detach().to("cpu", torch.float32)
        self.out_f, self.in_f = bw.shape
        if g.shape != (self.in_f, self.N_KNOTS) or sw.shape != (self.out_f, self.in_f, self.N_KNOTS - 4):
            raise ValueError("KANLinear with grid_size 5 and spline_order 3 expected")
        scaled = sw * ss.unsqueeze(-1)                    # scaled_spline_weight (kan.py:176-183)
        # k-major [in][1 + nb][out] (fac_kan_linear)
        self.wcat = torch.cat([bw.unsqueeze(-1), scaled], dim=2).permute(1, 2, 0).contiguous().to(device)
        self.grid = g.contiguous().to(device)
        self._scratch = None

    def __call__(self, x: torch.Tensor) -> torch.Tensor:
        rows = x.shape[0]
        lib = _lib.load()
        nbytes = lib.fac_kan_scratch_bytes(rows, self.in_f, self.out_f)
        if self._scratch is None or self._scratch.numel() * 4 < nbytes or self._scratch.device != x.device:
            self._scratch = torch.empty((nbytes + 3) // 4, dtype=torch.float32, device=x.device)
        y = torch.empty(rows, self.out_f, dtype=torch.float32, device=x.device)
        x = x.contiguous()
        _lib.check(lib.fac_kan_linear(x.data_ptr(), rows, self.in_f, self.out_f, self.grid.data_ptr(), self.N_KNOTS,
                                      self.wcat.data_ptr(), y.data_ptr(), self._scratch.data_ptr(), _stream(x)),
                   None, "fac_kan_linear")
        return y


def sigmoid(x: torch.Tensor) -> torch.Tensor:
    y = torch.empty_like(x)
    _lib.check(_lib.load().fac_sigmoid(x.data_ptr(), y.data_ptr(), x.numel(), _stream(x)), None, "fac_sigmoid")
    return y
