"""Drop-in ``S3D`` (BASELINE config 4) on gfx950 HIP kernels.

Mirrors ``sx_exp_deepfakedetect-master/S3D/model.py::S3D`` (:6-48): the same
constructor ``S3D(num_class, SRM_net)``, the same 465-key ``state_dict``
(``SRM.hpf``, ``base.{0..15}`` with BasicConv3d / SepConv3d / Mixed_* blocks,
``fc.0``) and ``forward(x)`` on a raw clip ``[B, 3, T, H, W]`` (0..255 BGR
floats, un-normalised — S3D-test.py:94-96) returning logits ``[B, num_class]``.

Arithmetic (every layer a HIP kernel of libfac_cvit.so, no CPU fallback):

* each Conv3d + BatchNorm3d(eval, eps 1e-3) + ReLU is one ``fac_conv_nd``
  implicit-GEMM launch with the BN folded on the host; SepConv3d is its
  (1,k,k) spatial and (k,1,1) temporal convs; the Inception branches write
  straight into their channel slot of the block output (no concat copy);
* MaxPool3d / the final avg_pool3d are ``fac_pool_nd``;
* the SRM high-pass bank (``SRM_net == 'yes'``, SRM/HPF.py) is a 3 -> 30
  (1,5,5) conv without BN or ReLU, written into a 32-channel buffer;
* ``fc`` (1x1x1 conv with bias) writes fp32 logits.  ``avg_pool3d((2, H, W),
  stride=1)`` then ``torch.mean`` over time is evaluated as two average pools
  before ``fc`` (identical in exact arithmetic: fc is affine).
"""
from __future__ import annotations

import math

import torch
from torch import nn

from . import _lib
from .cvit import _Node, weight_versions
from . import ops
from .ops import TORCH16, ConvLayer, conv_split, fold_bn, max_pool_sep, pack_input, pack_input_s2d, pool, s2d_weight, sigmoid
from .weights import s3d_base, s3d_param_specs

BN_EPS = 1e-3   # BatchNorm3d(eps=1e-3) in BasicConv3d / SepConv3d (model.py:54,67,71)
_BUFFERS = ("rmean", "rvar", "nbt")


def _pad_rows(t: torch.Tensor, n: int) -> torch.Tensor:
    """t with zero rows appended along dim 0 up to n rows."""
    if t.shape[0] == n:
        return t
    return torch.cat([t, t.new_zeros((n - t.shape[0],) + tuple(t.shape[1:]))])


def _init_tensor(shape, kind):
    if kind == "nbt":
        return torch.zeros((), dtype=torch.long)
    if kind in ("rmean", "beta", "lbias"):
        return torch.zeros(shape)
    if kind in ("rvar", "gamma"):
        return torch.ones(shape)
    t = torch.empty(shape)
    bound = 1.0 / math.sqrt(int(math.prod(shape[1:])))
    return t.uniform_(-bound, bound)


class S3D(nn.Module):
    def __init__(self, num_class: int, SRM_net: str, *, dtype: str = "fp16"):
        super().__init__()
        if dtype not in _lib.DTYPES:
            raise ValueError(f"dtype must be one of {list(_lib.DTYPES)}")
        self.num_class = num_class
        self.SRM_net = SRM_net
        self.dtype_name = dtype
        self._srm = SRM_net == "yes"
        # base.0 of a uint8 16 x 112 x 112 clip as one launch (ops.s3d_base0_u8)
        self.fuse_base0 = True
        for name, shape, kind in s3d_param_specs(num_class, self._srm):
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
        self.eval()

    def _versions(self):
        return weight_versions(self)

    def load_state_dict(self, state_dict, strict: bool = True, assign: bool = False):
        out = super().load_state_dict(state_dict, strict=strict, assign=assign)
        self._prep = None
        return out

    def train(self, mode: bool = True):
        if mode:
            raise RuntimeError("the gfx950 S3D path is inference-only (BatchNorm is folded into the convs)")
        return super().train(False)

    # ------------------------------------------------------------------ weights
    def _prepare(self, device: torch.device):
        idx = device.index if device.index is not None else torch.cuda.current_device()
        v = self._versions()
        if self._prep == (idx, v):
            return
        sd = self.state_dict()
        dt = self.dtype_name

        def bconv(p, stride=1, pad=0, cin_pad=None, kind="basic", cout_pad=None):
            ck, bn = (f"{p}.conv", f"{p}.bn") if kind == "basic" else (f"{p}.conv_{kind}", f"{p}.bn_{kind}")
            w, b = fold_bn(sd[ck + ".weight"], None, sd[bn + ".weight"], sd[bn + ".bias"], sd[bn + ".running_mean"],
                           sd[bn + ".running_var"], BN_EPS)
            if cout_pad:   # zero output channels (relu(0) = 0) up to cout_pad
                w, b = _pad_rows(w, cout_pad), _pad_rows(b, cout_pad)
            return ConvLayer(w, b, stride, pad, dtype=dt, device=device, cin_pad=cin_pad)

        def sep(p, k, s, pd, cin_pad=None, mid_pad=None):
            # mid_pad: the (1,k,k) half's output (the (k,1,1) half's input)
            # zero-padded to mid_pad channels
            return (bconv(p, (1, s, s), (0, pd, pd), cin_pad, "s", cout_pad=mid_pad),
                    bconv(p, (s, 1, 1), (pd, 0, 0), mid_pad, "t"))

        def sep_s2d(p):
            # base.0 without SRM: the (1,7,7)/(1,2,2) 3-channel conv as a (1,4,4)/1 conv over
            # space-to-depth cells of each frame (ops.pack_input_s2d / s2d_weight)
            w, b = fold_bn(sd[p + ".conv_s.weight"], None, sd[p + ".bn_s.weight"], sd[p + ".bn_s.bias"],
                           sd[p + ".bn_s.running_mean"], sd[p + ".bn_s.running_var"], BN_EPS)
            return (ConvLayer(s2d_weight(w), b, 1, 0, dtype=dt, device=device),
                    bconv(p, (2, 1, 1), (3, 0, 0), None, "t"))

        self._srm_conv = None
        if self._srm:
            w = sd["SRM.hpf.weight"]
            self._srm_conv = ConvLayer(w, torch.zeros(w.shape[0]), 1, (0, 2, 2), dtype=dt, device=device)
        self._layers = []
        for i, L in enumerate(s3d_base(self._srm)):
            p = f"base.{i}"
            if L[0] == "sep" and i == 0 and not self._srm:
                self._layers.append(("sep_s2d", sep_s2d(p)))
            elif L[0] == "sep":
                self._layers.append(("sep", sep(p, L[3], L[4], L[5], cin_pad=32 if i == 0 else None)))
            elif L[0] == "basic":
                self._layers.append(("basic", bconv(p)))
            elif L[0] == "pool":
                self._layers.append(("pool", L[1:]))
            else:
                cin, b0, (b1a, b1b), (b2a, b2b), b3 = L[1:]
                # the three 1x1x1 heads reading the block input (branch0.0,
                # branch1.0, branch2.0) also as ONE conv over their
                # concatenated output channels (ops.conv_split)
                heads = [fold_bn(sd[f"{h}.conv.weight"], None, sd[f"{h}.bn.weight"], sd[f"{h}.bn.bias"],
                                 sd[f"{h}.bn.running_mean"], sd[f"{h}.bn.running_var"], BN_EPS)
                         for h in (f"{p}.branch0.0", f"{p}.branch1.0", f"{p}.branch2.0")]
                merged = ConvLayer(torch.cat([h[0] for h in heads]), torch.cat([h[1] for h in heads]), 1, 0,
                                   dtype=dt, device=device)
                # merged path below 14x14 (no conv.hip tile there): branch1.0 /
                # branch2.0 outputs padded with zero channels to a multiple of
                # 64 (zero weight rows and biases: relu(0) = 0), so the (1,3,3)
                # convs reading them take K steps that each lie in one tap
                # (convnd_igemm's uniform-tap gather)
                p1, p2 = self._pad64(b1a, 1), self._pad64(b2a, 2)
                # and (padt) the SepConvs' middle channels, so their
                # (3,1,1) halves take the uniform-tap gather too
                m1 = (b1b + 63) // 64 * 64 if self.padt else b1b
                m2 = (b2b + 63) // 64 * 64 if self.padt else b2b
                # at 14x14 and above, branch2's SepConv middle channels 96 ->
                # 128 (zero rows of the (1,3,3) half): that half then has a
                # conv.hip tile and the (3,1,1) half reads a uniform-tap K
                # (convnd_pt with a partial column block). Mixed_3c, 384 clips:
                # 327 -> 160 us (tools/archive/s3d_small_ab.py); 32 -> 64 is slower
                m2w = (b2b + 127) // 128 * 128 if b2b > 64 and b2b % 64 else None
                b1, b2 = sep(f"{p}.branch1.1", 3, 1, 1), sep(f"{p}.branch2.1", 3, 1, 1, mid_pad=m2w)

                def padded(p=p, heads=heads, merged=merged, b1=b1, b2=b2, b1a=b1a, b1b=b1b, b2a=b2a, b2b=b2b,
                           p1=p1, p2=p2, m1=m1, m2=m2):
                    # the channel-padded layers, built on the block's first
                    # forward below 14x14 (never for the larger
                    # blocks, whose padded copies no launch reads)
                    merged_p = merged
                    if (p1, p2) != (b1a, b2a):
                        hw = [heads[0][0], _pad_rows(heads[1][0], p1), _pad_rows(heads[2][0], p2)]
                        hb = [heads[0][1], _pad_rows(heads[1][1], p1), _pad_rows(heads[2][1], p2)]
                        merged_p = ConvLayer(torch.cat(hw), torch.cat(hb), 1, 0, dtype=dt, device=device)
                    return dict(
                        b1p=b1 if (p1, m1) == (b1a, b1b) else sep(f"{p}.branch1.1", 3, 1, 1, cin_pad=p1, mid_pad=m1),
                        b2p=b2 if (p2, m2) == (b2a, b2b) else sep(f"{p}.branch2.1", 3, 1, 1, cin_pad=p2, mid_pad=m2),
                        heads_p=merged_p)
                self._layers.append(("mixed", dict(
                    b1=b1, b2=b2, b3=bconv(f"{p}.branch3.1"), padded=padded,
                    heads=merged, head_splits=(b0, b0 + b1a), head_widths=(b1a, b2a),
                    head_splits_p=(b0, b0 + p1), head_widths_p=(p1, p2),
                    widths=(b0, b1b, b2b, b3))))
        self._fc = ConvLayer(sd["fc.0.weight"], sd["fc.0.bias"], 1, 0, dtype=dt, device=device)
        self._prep = (idx, v)

    # ------------------------------------------------------------------ forward
    # channel padding of the merged heads' branch1.0 / branch2.0 outputs to a
    # multiple of 64: 0 none, 1 branch1.0 when >= 64 channels, 2 both
    # (level 1 measured fastest); and the SepConvs' middle channels to a
    # multiple of 64 (padt), so their (3,1,1) halves take the uniform-tap gather
    pad64_level = 1
    padt = True
    # branch3's MaxPool3d(3, 1, 1) fused into its 1x1x1 conv (FAC_CONV_MAXPOOL3S1)
    # on the 14 / 7 / 3 maps; False: fac_pool_nd then the conv (A/B)
    fuse_pool3 = True
    # base.1's pool fused into base.2's 1x1x1 conv (FAC_CONV_PREPOOL3S2) on
    # 56-wide maps; False: fac_pool_nd then the conv (A/B)
    fuse_pool1 = True
    # Mixed_3b's / 3c's branch2 SepConv (16 -> 32 -> 32 / 32 -> 96 -> 96 on
    # 8 x 14 x 14) as one launch (fac_sep_tiny / fac_sep_mid); False: the two
    # fac_conv_nd launches (A/B)
    fuse_sep = True

    def _pad64(self, c: int, level: int) -> int:
        if self.pad64_level < level or c % 64 == 0 or (level == 1 and c < 64):
            return c
        return (c + 63) // 64 * 64

    def _mixed(self, x, blk):
        """One Mixed_* block (model.py:84-342).  Its four branches read the
        same input and write disjoint channel slots of the block output: the
        three 1x1x1 heads (branch0.0, branch1.0, branch2.0) as one
        column-split launch (ops.conv_split: branch0 straight into its slot),
        then branch1's and branch2's SepConvs, then branch3's MaxPool3d(3,1,1)
        + 1x1x1 (one launch where maxpool3_pw covers the map: the pooled map
        never goes through memory).  (The branches on concurrent side streams measured faster or
        slower depending on which hardware queues torch's pool streams land on
        -- 27.0k vs 20.5k clips/s for the same graph -- so the serial order is
        the dependable one.)"""
        n, d, h, w, _ = x.shape
        out = torch.empty(n, d, h, w, sum(blk["widths"]), dtype=x.dtype, device=x.device)
        o1 = blk["widths"][0]
        o2 = o1 + blk["widths"][1]
        o3 = o2 + blk["widths"][2]
        sfx = "_p" if h < 14 else ""   # channel-padded heads (pad64_level) where no conv.hip tile exists
        if sfx and "heads_p" not in blk:
            if torch.cuda.is_current_stream_capturing():
                raise RuntimeError("S3D: run one eager forward at this clip size before graph capture "
                                   "(the padded late-block layers are built on first use)")
            blk.update(blk["padded"]())
        s1, t1 = blk["b1p" if sfx else "b1"]
        s2, t2 = blk["b2p" if sfx else "b2"]
        hws = blk["head_widths" + sfx]
        h1 = torch.empty(n, d, h, w, hws[0], dtype=x.dtype, device=x.device)
        h2 = torch.empty(n, d, h, w, hws[1], dtype=x.dtype, device=x.device)
        conv_split(blk["heads" + sfx], x, blk["head_splits" + sfx], out, 0, h1, h2)
        t1(s1(h1), out=out, c_off=o1)
        if self.fuse_sep and (ops.sep_tiny_ok(s2, t2, h2) or ops.sep_mid_ok(s2, t2, h2)):
            ops.sep_tiny(s2, t2, h2, out, o2)   # Mixed_3b's / 3c's branch2 SepConv in one launch
        else:
            t2(s2(h2), out=out, c_off=o2)
        b3 = blk["b3"]
        if self.fuse_pool3 and b3.maxpool3s1_ok(x, out, o3):
            b3(x, out=out, c_off=o3, maxpool3s1=True)       # pool + 1x1x1 in one launch (ops.hip maxpool3_pw)
        else:
            b3(max_pool_sep(x, 3, 1, 1), out=out, c_off=o3)
        return out

    def features16(self, x16: torch.Tensor, taps: list | None = None) -> torch.Tensor:
        """`base` (model.py:17-33) on the packed clip (`_pack`: without SRM the
        raw fp32 clip, or its ops.pack_input_s2d cells) -> [B, T', H', W', 1024] 16-bit.
        With `taps`, the output of every base[i] ([B, T, H, W, C] channels-last,
        16-bit) is appended to it, in order."""
        y = x16
        if self._srm_conv is not None:
            n, d, h, w, _ = y.shape
            s = torch.zeros(n, d, h, w, 32, dtype=y.dtype, device=y.device)   # 30 filters + 2 zero channels
            y = self._srm_conv(y, relu=False, out=s)
        skip = False
        for li, (kind, L) in enumerate(self._layers):
            if skip:   # base.2, run with base.1's pool below
                skip = False
                continue
            nxt = self._layers[li + 1] if li + 1 < len(self._layers) else (None, None)
            if (kind == "pool" and self.fuse_pool1 and L == ((1, 3, 3), (1, 2, 2), (0, 1, 1)) and nxt[0] == "basic"
                    and taps is None and nxt[1].prepool3s2_ok(y)):   # (taps: base.1's own output is one)
                # base.1's MaxPool3d((1,3,3),(1,2,2)) + base.2's 1x1x1 conv as one
                # launch (FAC_CONV_PREPOOL3S2, ops.hip maxpool2s_pw)
                y = nxt[1](y, prepool3s2=True)
                skip = True
                continue
            if kind == "sep_s2d":
                # the raw clip (`_pack`): the space-to-depth packing runs
                # inside the conv's halo staging (ops.conv_s2d4_clip); packed
                # cells (ops.pack_input_s2d) still take the plain conv.  A
                # uint8 16 x 112 x 112 clip runs both halves as one launch
                # (ops.s3d_base0_u8; fuse_base0 = False: the two launches)
                if y.dtype == torch.uint8 and self.fuse_base0 and tuple(y.shape[2:]) == (16, 112, 112) and \
                        _lib.exports("fac_s3d_base0_u8"):
                    y = ops.s3d_base0_u8(L[0], L[1], y)
                else:
                    y = L[1](ops.conv_s2d4_clip(L[0], y) if y.dtype in (torch.float32, torch.uint8) else L[0](y))
            elif kind == "sep":
                y = L[1](L[0](y))
            elif kind == "basic":
                y = L(y)
            elif kind == "pool":
                y = max_pool_sep(y, *L)
            else:
                y = self._mixed(y, L)
            if taps is not None:
                taps.append(y)
        return y

    def _pack(self, x: torch.Tensor) -> torch.Tensor:
        if not x.is_cuda:
            raise RuntimeError("S3D (gfx950 HIP path) needs its input on a GPU device; there is no CPU fallback")
        if x.dim() != 5 or x.shape[1] != 3:
            raise ValueError(f"expected a clip [B,3,T,H,W], got {tuple(x.shape)}")
        self._prepare(x.device)
        _, _, T, H, W = x.shape
        if self._srm:
            return pack_input(x.float(), dtype=self.dtype_name, u8=False, spatial=(T, H, W))
        # base.0's space-to-depth cells are made inside its conv (ops.conv_s2d4_clip);
        # a uint8 clip (decoded frames: the reference's values before its float
        # cast, S3D-test.py:94-96) is read as is, a quarter of the bytes.  That
        # kernel tiles the output in 8 x 28 boxes of the half-resolution map
        # (H % 16 == 0, W % 56 == 0, e.g. 112 x 112 or 224 x 224); any other
        # size (the reference takes any: avg_pool3d runs over the full map,
        # model.py:43) gets packed cells and base.0 runs on the generic conv.
        if H % 16 == 0 and W % 56 == 0:
            if x.dtype == torch.uint8 and _lib.exports("fac_conv_s2d4_clip_u8"):
                return x.contiguous()
            if _lib.exports("fac_conv_s2d4_clip"):
                return x.float().contiguous()
        return pack_input_s2d(x.float(), dtype=self.dtype_name, u8=False, pad_before=2, pad_after=1)

    def base_outputs(self, x: torch.Tensor) -> list:
        """The output of every base[i] (model.py:17-33) for the raw clip `x`,
        channels-last 16-bit: what a forward hook on the reference's
        ``base[i]`` sees, for per-block parity checks."""
        taps = []
        self.features16(self._pack(x), taps)
        return taps

    def forward(self, x: torch.Tensor, return_probs: bool = False):
        x16 = self._pack(x)
        B = x.shape[0]
        y = self.features16(x16)
        _, t, h, w, _ = y.shape
        y = pool(y, (2, h, w), 1, 0, "avg")                           # F.avg_pool3d(y, (2, H, W), stride=1)
        y = pool(y, (y.shape[1], 1, 1), 1, 0, "avg")                  # torch.mean over time (before fc: affine)
        logits = self._fc(y, relu=False, out_f32=True).view(B, self.num_class)
        return (logits, sigmoid(logits)) if return_probs else logits


def custom_round(values):
    """utils.py:25-32: 1 where a value is > 0.5, else 0."""
    return (torch.as_tensor(values, dtype=torch.float64) > 0.5).to(torch.int64).numpy()


def custom_video_round(preds):
    """utils.py:34-38: the first value > 0.5, else the mean."""
    for p in preds:
        if p > 0.5:
            return p
    return sum(preds) / len(preds)


def video_predictions(model: S3D, snippets: torch.Tensor, batch: int = 64) -> list:
    """The per-video score of S3D-test.py's modeleval (:259-283) for a batch of
    videos, one snippet each (read_frames keeps every 10th of the first 200
    frames: one [3, 20, H, W] snippet per video, :185-195), as a list of
    floats.  Per video the reference takes ``sigmoid`` of each row of the
    model's output, their mean, element [0] (:269-276), and
    ``custom_video_round`` only when a video has more than one face
    prediction, which one snippet never has (:280-283).  Snippets run through
    the drop-in in batches of `batch` clips; each video's logits are
    independent of its batch neighbours."""
    if snippets.dim() != 5:
        raise ValueError(f"expected snippets [V,3,T,H,W], got {tuple(snippets.shape)}")
    out = []
    for v0 in range(0, snippets.shape[0], batch):
        _, probs = model(snippets[v0:v0 + batch], return_probs=True)
        for p in probs.double().cpu():
            faces_preds = [p]                                   # one snippet = one prediction row
            cur = sum(faces_preds) / len(faces_preds)
            video_faces_preds = [float(cur[0])]
            out.append(custom_video_round(video_faces_preds) if len(video_faces_preds) > 1
                       else video_faces_preds[0])
    return out


__all__ = ["S3D", "TORCH16", "custom_round", "custom_video_round", "video_predictions"]
