"""Layer kernels of include/fac_ops.h and the ResVitKan drop-in on the GPU.

* fac_conv_nd vs a plain PyTorch fp32 convolution (CPU) of the same 16-bit
  operands: bit-equal after rounding except for accumulation-order flips of
  one 16-bit ulp (<= 1 ulp everywhere, on <= 5% of the outputs) — over 2-D and
  3-D kernels, strides, paddings, ragged channel counts, fp32 output, concat
  offsets and the Bottleneck residual epilogue.
* fac_pool_nd: bit-exact (max) / within fp32 rounding of one 16-bit ulp (avg).
* fac_kan_linear vs the reference's KANLinear outputs (golden): <= 1e-5.
* ResVitKan forward vs the reference module's logits (golden, fp32):
  per-logit sigmoid within 1e-3 with fp16 operands and, with bf16, within
  1.25x the oracle's emulated bf16 envelope on the same inputs (1.9e-3 for
  ResVitKan, 0.8-1.0e-3 for S3D: tests/golden/bf16_envelope.json) plus 5e-4
  for the fp32 summation order (conftest.bf16_gate).
"""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from fac_fake_amd.weights import make_crops, make_resvitkan_state_dict

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
T16 = {"bf16": torch.bfloat16, "fp16": torch.float16}


def _ulps(a: torch.Tensor, b: torch.Tensor, dt: str) -> torch.Tensor:
    """|a - b| in units of the 16-bit ulp at max(|a|, |b|), after allowing the
    fp32 accumulation noise of a K-term dot product (2^-16 of the output
    scale: outputs that are the small difference of O(1) partial sums carry
    fp32 rounding a few fp16 ulps of their own size)."""
    a, b = a.float(), b.float()
    m = torch.maximum(a.abs(), b.abs()).clamp_min(1e-30)
    e = torch.floor(torch.log2(m))
    ulp = torch.pow(2.0, e - (7 if dt == "bf16" else 10))
    if dt == "fp16":
        ulp = ulp.clamp_min(2.0 ** -24)   # fp16 subnormals: fixed spacing
    noise = 2.0 ** -16 * torch.maximum(a.abs().max(), b.abs().max())
    return ((a - b).abs() - noise).clamp_min(0) / ulp


CONV_CASES = [
    # (n, d, h, w, cin, cout, k(kd,kh,kw), stride, pad)
    (2, 1, 17, 19, 64, 64, (1, 1, 1), 1, 0),
    (2, 1, 14, 14, 64, 200, (1, 3, 3), 1, (0, 1, 1)),
    (2, 1, 15, 15, 128, 96, (1, 3, 3), (1, 2, 2), (0, 1, 1)),
    (1, 1, 40, 40, 8, 64, (1, 7, 7), (1, 2, 2), (0, 3, 3)),
    (2, 1, 9, 9, 256, 512, (1, 1, 1), (1, 2, 2), 0),
    (1, 6, 10, 10, 16, 32, (3, 1, 1), 1, (1, 0, 0)),
    (1, 5, 12, 12, 24, 48, (1, 3, 3), 1, (0, 1, 1)),
    (1, 8, 16, 16, 8, 64, (3, 7, 7), 2, (1, 3, 3)),
    (1, 3, 7, 7, 40, 12, (1, 1, 1), 1, 0),
    # 3x3/1 convs routed to conv.hip's halo kernel (ResNet-50 / S3D widths)
    (2, 1, 56, 56, 64, 64, (1, 3, 3), 1, (0, 1, 1)),
    (1, 2, 28, 28, 64, 192, (1, 3, 3), 1, (0, 1, 1)),
    (2, 1, 28, 28, 128, 128, (1, 3, 3), 1, (0, 1, 1)),
    (2, 1, 14, 14, 256, 256, (1, 3, 3), 1, (0, 1, 1)),
    # S3D's temporal convs with 8 output frames (ops.hip conv_tk)
    (2, 16, 8, 8, 64, 64, (7, 1, 1), (2, 1, 1), (3, 0, 0)),
    (2, 8, 4, 8, 192, 192, (3, 1, 1), 1, (1, 0, 0)),
    (2, 8, 7, 9, 64, 128, (3, 1, 1), 1, (1, 0, 0)),           # 63 positions: partial last unit
    (1, 16, 14, 14, 192, 64, (7, 1, 1), (2, 1, 1), (3, 0, 0)),  # 196 positions
    # the space-to-depth first conv (ops.hip conv_s2d4: 4x4/1, 16 -> 64, 8 x 28 boxes)
    (2, 2, 19, 31, 16, 64, (1, 4, 4), 1, 0),
    (1, 1, 59, 59, 16, 64, (1, 4, 4), 1, 0),
    # stride-1 1x1 convs with cin 64 / 128 / 256 (ops.hip conv_pw; case 0 too)
    (3, 1, 23, 29, 128, 192, (1, 1, 1), 1, 0),
    (1, 1, 56, 56, 64, 256, (1, 1, 1), 1, 0),
    (2, 1, 14, 15, 256, 128, (1, 1, 1), 1, 0),
    # cin % 64 == 0 on convnd_igemm: the uniform-tap gather (one tap per K step)
    (2, 4, 9, 11, 64, 128, (3, 3, 3), 1, 1),                 # 3-D taps, padding on every axis
    (2, 3, 7, 7, 192, 130, (3, 3, 3), (1, 2, 2), (1, 1, 1)),  # ragged cout, strided
    (4, 1, 112, 256, 320, 128, (1, 1, 1), 1, 0),            # M = 114688: the 256 x 128 tile
]


@pytest.mark.parametrize("dt", ["bf16", "fp16"])
@pytest.mark.parametrize("case", range(len(CONV_CASES)))
def test_conv_nd_vs_torch_fp32(case, dt):
    from fac_fake_amd.ops import ConvLayer
    n, d, h, w, cin, cout, k, st, pd = CONV_CASES[case]
    g = torch.Generator().manual_seed(100 + case)
    x = torch.randn(n, cin, d, h, w, generator=g).to(T16[dt]).float()
    wt = (torch.randn(cout, cin, *k, generator=g) / np.sqrt(cin * np.prod(k))).float()
    b = torch.randn(cout, generator=g) * 0.1
    layer = ConvLayer(wt, b, st, pd, dtype=dt, device=DEV)
    xg = x.permute(0, 2, 3, 4, 1).contiguous().to(T16[dt]).to(DEV)
    y = layer(xg, relu=True)
    torch.cuda.synchronize()
    ref = F.relu(F.conv3d(x, wt.to(T16[dt]).float(), b, stride=st, padding=pd)).permute(0, 2, 3, 4, 1)
    yr = ref.to(T16[dt])
    u = _ulps(y.cpu(), yr, dt)
    assert tuple(y.shape) == tuple(yr.shape)
    assert u.max() <= 1.0, (case, float(u.max()))
    assert (u > 0).float().mean() <= 0.05


@pytest.mark.parametrize("dt", ["bf16", "fp16"])
@pytest.mark.parametrize("shape,cin", [((2, 28, 28), 192), ((3, 7, 9), 192), ((1, 14, 14), 192),
                                       ((2, 14, 14), 128), ((3, 7, 9), 128)])
def test_conv_tk2_weights_in_vgprs_bit_identical(shape, cin, dt):
    """S3D's cin-192 / 128 (3,1,1) temporal convs (base.3 / Mixed_3b-3c conv_t,
    model.py:63-82) with each wave's weight fragments in VGPRs
    (fac_set_option "tk_wreg" 1, the default) against the same kernel reading
    them from LDS ("tk_wreg" 0): the same MFMA order, so bit-identical, and
    within one 16-bit ulp of PyTorch fp32.  (3, 7, 9): 63 positions, a partial
    last 16-position unit."""
    from fac_fake_amd.ops import ConvLayer
    n, h, w = shape
    g = torch.Generator().manual_seed(5 + h * w + cin)
    x = torch.randn(n, cin, 8, h, w, generator=g).to(T16[dt]).float()
    wt = torch.randn(cin, cin, 3, 1, 1, generator=g) / np.sqrt(3 * cin)
    b = torch.randn(cin, generator=g) * 0.1
    layer = ConvLayer(wt, b, 1, (1, 0, 0), dtype=dt, device=DEV)
    xg = x.permute(0, 2, 3, 4, 1).contiguous().to(T16[dt]).to(DEV)
    outs = {}
    try:
        for v in (1, 0):
            _set_knob(b"tk_wreg", v, dt)
            outs[v] = layer(xg, relu=True)
            torch.cuda.synchronize()
            outs[v] = outs[v].cpu()
    finally:
        _set_knob(b"tk_wreg", 1, dt)
    assert torch.equal(outs[1], outs[0])
    ref = F.relu(F.conv3d(x, wt.to(T16[dt]).float(), b, padding=(1, 0, 0))).permute(0, 2, 3, 4, 1).to(T16[dt])
    u = _ulps(outs[1], ref, dt)
    assert u.max() <= 1.0 and (u > 0).float().mean() <= 0.05


def _nd_pt_wide(value: int, dt: str):
    """fac_set_option("nd_pt_wide") is process-wide; any context sets it."""
    import ctypes
    from fac_fake_amd import _lib
    lib = _lib.load()
    h = ctypes.c_void_p()
    _lib.check(lib.fac_create(0, _lib.DTYPES[dt], ctypes.byref(h)), None, "fac_create")
    try:
        _lib.check(lib.fac_set_option(h, b"nd_pt_wide", value), h, "fac_set_option")
    finally:
        lib.fac_destroy(h)


@pytest.mark.parametrize("dt", ["bf16", "fp16"])
@pytest.mark.parametrize("n,d,h,w,cin,cout,k,pd,c_off", [
    (2, 8, 14, 14, 128, 96, (3, 1, 1), (1, 0, 0), 0),      # S3D Mixed_3c branch2 (3,1,1) half, mid padded
    (3, 1, 23, 29, 192, 32, (1, 1, 1), 0, 8),              # cout 32 into a channel slot of a wider tensor
    (2, 3, 7, 7, 128, 200, (1, 3, 3), (0, 1, 1), 0),       # two column blocks, the second 72 wide
    (1, 5, 9, 13, 64, 136, (3, 3, 3), 1, 16),              # 3-D taps, partial row tile, c_off
])
def test_conv_nd_pt_partial_column_block(n, d, h, w, cin, cout, k, pd, c_off, dt):
    """convnd_pt with cout % 128 != 0 (a partial last column block whose
    padding channels store into a sink, so the hand-counted vmcnt waits still
    see every store): forced onto these small shapes with nd_pt_wide = 1 (any
    row-tile count), against torch's fp32 conv (one 16-bit ulp) and against
    the convnd_igemm route (nd_pt_wide = 0), and the channels around the
    written slot left untouched."""
    from fac_fake_amd.ops import ConvLayer
    g = torch.Generator().manual_seed(cin + cout)
    x = torch.randn(n, cin, d, h, w, generator=g).to(T16[dt]).float()
    wt = (torch.randn(cout, cin, *k, generator=g) / np.sqrt(cin * np.prod(k))).float()
    b = torch.randn(cout, generator=g) * 0.1
    layer = ConvLayer(wt, b, 1, pd, dtype=dt, device=DEV)
    xg = x.permute(0, 2, 3, 4, 1).contiguous().to(T16[dt]).to(DEV)
    od, oh, ow = layer.out_dims(d, h, w)
    outs = {}
    try:
        for v in (1, 0):
            _nd_pt_wide(v, dt)
            o = torch.full((n, od, oh, ow, c_off + cout + 8), 7.0, device=DEV, dtype=T16[dt])
            layer(xg, relu=True, out=o, c_off=c_off)
            torch.cuda.synchronize()
            outs[v] = o.cpu()
    finally:
        _nd_pt_wide(32, dt)
    y = outs[1]
    assert torch.all(y[..., :c_off] == 7.0) and torch.all(y[..., c_off + cout:] == 7.0)
    ref = F.relu(F.conv3d(x, wt.to(T16[dt]).float(), b, padding=pd)).permute(0, 2, 3, 4, 1)
    u = _ulps(y[..., c_off:c_off + cout], ref.to(T16[dt]), dt)
    assert u.max() <= 1.0 and (u > 0).float().mean() <= 0.05
    u2 = _ulps(y, outs[0], dt)
    assert u2.max() <= 1.0 and (u2 > 0).float().mean() <= 0.05


@pytest.mark.parametrize("dt", ["bf16", "fp16"])
@pytest.mark.parametrize("cin,cmid,n1,hw", [(64, 256, 64, (56, 56)), (64, 256, 128, (23, 29)),
                                            (128, 512, 128, (28, 28)), (128, 512, 128, (13, 11))])
def test_bottleneck_pw2_matches_two_launches(cin, cmid, n1, hw, dt):
    """fac_bottleneck_pw2 (a layer1 bottleneck's conv3 + identity residual and
    the next block's conv1 in one launch) against the two separate
    fac_conv_nd launches it replaces: the block output within one 16-bit ulp
    on <= 5% of elements (fp32 summation order), the conv1 output within one
    ulp of torch's fp32 conv of the fused kernel's own block output.  Layer1
    (64 -> 256 -> 64 / 128, bneck_pw2) and layer2 (128 -> 512 -> 128,
    bneck_pw2_l2) shapes; 29x23 and 13x11 positions leave a partial last row
    tile."""
    from fac_fake_amd.ops import ConvLayer, bottleneck_pw2
    g = torch.Generator().manual_seed(5 + n1)
    n = 3
    h = torch.randn(n, 1, *hw, cin, generator=g).relu().to(T16[dt])
    res = torch.randn(n, 1, *hw, cmid, generator=g).relu().to(T16[dt])
    w3, b3 = torch.randn(cmid, cin, 1, 1, 1, generator=g) / np.sqrt(cin), torch.randn(cmid, generator=g) * 0.1
    w1, b1 = torch.randn(n1, cmid, 1, 1, 1, generator=g) / np.sqrt(cmid), torch.randn(n1, generator=g) * 0.1
    c3 = ConvLayer(w3, b3, 1, 0, dtype=dt, device=DEV)
    c1 = ConvLayer(w1, b1, 1, 0, dtype=dt, device=DEV)
    hg, rg = h.to(DEV), res.to(DEV)
    x, h1 = bottleneck_pw2(c3, hg, rg, c1)
    xr = c3(hg, residual=rg, relu2=True)
    h1r = c1(xr)
    torch.cuda.synchronize()
    u = _ulps(x.cpu(), xr.cpu(), dt)
    assert u.max() <= 1.0 and (u > 0).float().mean() <= 0.05
    if torch.equal(x.cpu(), xr.cpu()):
        u1 = _ulps(h1.cpu(), h1r.cpu(), dt)
        assert u1.max() <= 1.0 and (u1 > 0).float().mean() <= 0.05
    ref1 = F.relu(F.conv3d(x.cpu().float().permute(0, 4, 1, 2, 3), w1.to(T16[dt]).float(), b1))
    u2 = _ulps(h1.cpu(), ref1.permute(0, 2, 3, 4, 1).to(T16[dt]), dt)
    assert u2.max() <= 1.0 and (u2 > 0).float().mean() <= 0.05


@pytest.mark.parametrize("dt", ["bf16", "fp16"])
@pytest.mark.parametrize("n,t,relu", [(2, 3, True), (4, 10, False), (20, 8, True)])
def test_conv_s2d4_clip_equals_pack_then_conv(n, t, relu, dt):
    """fac_conv_s2d4_clip (S3D's base.0 spatial conv with the space-to-depth
    packing folded into the halo staging, fp32 clip in) against
    fac_pack_input_s2d + fac_conv_nd: bit-identical, for raw 0..255 clips,
    one box per workgroup (n*t*14 = 84 boxes), a few (560) and several (2240)
    boxes per persistent workgroup (the register prefetch of the next box's
    pixels and the double-buffered cells), with and without ReLU."""
    from fac_fake_amd.ops import ConvLayer, conv_s2d4_clip, pack_input_s2d, s2d_weight
    g = torch.Generator().manual_seed(n + t)
    clip = (torch.rand(n, 3, t, 112, 112, generator=g) * 255).to(DEV)
    wt = torch.randn(64, 3, 1, 7, 7, generator=g) / 12
    b = torch.randn(64, generator=g) * 0.5
    layer = ConvLayer(s2d_weight(wt), b, 1, 0, dtype=dt, device=DEV)
    fused = conv_s2d4_clip(layer, clip, relu=relu)
    ref = layer(pack_input_s2d(clip, dtype=dt, u8=False, pad_before=2, pad_after=1), relu=relu)
    torch.cuda.synchronize()
    assert tuple(fused.shape) == (n, t, 56, 56, 64)
    assert torch.equal(fused.view(torch.int16).cpu(), ref.view(torch.int16).cpu())
    # the uint8 clip (fac_conv_s2d4_clip_u8) equals the fp32 path on the same values
    clip8 = clip.to(torch.uint8)
    f8 = conv_s2d4_clip(layer, clip8, relu=relu)
    f32 = conv_s2d4_clip(layer, clip8.float(), relu=relu)
    torch.cuda.synchronize()
    assert torch.equal(f8.view(torch.int16).cpu(), f32.view(torch.int16).cpu())


@pytest.mark.parametrize("dt", ["bf16", "fp16"])
@pytest.mark.parametrize("n,d,h,w", [(2, 1, 19, 59), (1, 2, 35, 31), (3, 1, 115, 115), (300, 1, 19, 59)])
def test_conv_s2d4_maxpool_fused(n, d, h, w, dt):
    """conv_s2d4_mp (FAC_CONV_MAXPOOL3S2): the 4x4/1 space-to-depth conv +
    bias + ReLU + MaxPool2d(3, 2, 1) in one launch is bit-identical to
    conv_s2d4 followed by fac_pool_nd (a max selects one of its inputs, and
    rounding is monotone), and within one 16-bit ulp of torch's fp32 conv ->
    relu -> rounded -> max_pool.  Every box touches the top or left pool
    padding on the first row / column of boxes; biases straddle 0 so ReLU
    zeros occur.  300 images of 2 column strips each (600 > 2 x 256 CUs):
    each persistent workgroup walks several strips (the carry reset, the
    cross-strip halo prefetch and its counted waits)."""
    from fac_fake_amd.ops import ConvLayer, max_pool_sep
    g = torch.Generator().manual_seed(7 + h + d)
    x = torch.randn(n, 16, d, h, w, generator=g).to(T16[dt]).float()
    wt = (torch.randn(64, 16, 1, 4, 4, generator=g) / 16).float()
    b = torch.randn(64, generator=g) * 0.5
    layer = ConvLayer(wt, b, 1, 0, dtype=dt, device=DEV)
    xg = x.permute(0, 2, 3, 4, 1).contiguous().to(T16[dt]).to(DEV)
    fused = layer(xg, relu=True, maxpool3s2=True)
    unf = max_pool_sep(layer(xg, relu=True), (1, 3, 3), (1, 2, 2), (0, 1, 1))
    torch.cuda.synchronize()
    assert tuple(fused.shape) == (n, d, (h - 3) // 2, (w - 3) // 2, 64)
    assert torch.equal(fused.cpu(), unf.cpu())
    conv = F.relu(F.conv3d(x, wt.to(T16[dt]).float(), b)).to(T16[dt]).float()
    ref = F.max_pool3d(conv, (1, 3, 3), (1, 2, 2), (0, 1, 1)).permute(0, 2, 3, 4, 1).to(T16[dt])
    u = _ulps(fused.cpu(), ref, dt)
    assert u.max() <= 1.0 and (u > 0).float().mean() <= 0.05


@pytest.mark.parametrize("dt", ["bf16", "fp16"])
@pytest.mark.parametrize("cin,cout", [(64, 256), (128, 512), (256, 1024), (256, 64)])
def test_conv_pw_residual_into_slot(cin, cout, dt):
    """conv_pw's bottleneck epilogue relu(relu(conv + b) + res) written into
    a channel slot of a wider buffer, over enough positions (40 000, ragged
    last tile) that every persistent workgroup walks several row tiles."""
    from fac_fake_amd.ops import ConvLayer
    g = torch.Generator().manual_seed(11 + cin)
    n, h, w = 4, 100, 100
    x = torch.randn(n, cin, 1, h, w, generator=g).to(T16[dt]).float()
    wt = torch.randn(cout, cin, 1, 1, 1, generator=g) / np.sqrt(cin)
    b = torch.randn(cout, generator=g) * 0.1
    res = torch.randn(n, 1, h, w, cout, generator=g).to(T16[dt])
    layer = ConvLayer(wt, b, 1, 0, dtype=dt, device=DEV)
    big = torch.zeros(n, 1, h, w, cout + 16, dtype=T16[dt], device=DEV)
    xg = x.permute(0, 2, 3, 4, 1).contiguous().to(T16[dt]).to(DEV)
    layer(xg, relu=True, out=big, c_off=8, residual=res.to(DEV), relu2=True)
    torch.cuda.synchronize()
    conv = F.conv3d(x, wt.to(T16[dt]).float(), b).permute(0, 2, 3, 4, 1)
    ref = F.relu(F.relu(conv) + res.float()).to(T16[dt])
    bc = big.cpu()
    u = _ulps(bc[..., 8:8 + cout], ref, dt)
    assert u.max() <= 1.0 and (u > 0).float().mean() <= 0.05
    assert bc[..., :8].abs().max() == 0 and bc[..., 8 + cout:].abs().max() == 0


def _set_knob(name: bytes, value: int, dt: str):
    """A process-wide fac_set_option knob (any context sets it)."""
    import ctypes
    from fac_fake_amd import _lib
    lib = _lib.load()
    h = ctypes.c_void_p()
    _lib.check(lib.fac_create(0, _lib.DTYPES[dt], ctypes.byref(h)), None, "fac_create")
    try:
        _lib.check(lib.fac_set_option(h, name, value), h, "fac_set_option")
    finally:
        lib.fac_destroy(h)


@pytest.mark.parametrize("dt", ["bf16", "fp16"])
@pytest.mark.parametrize("n,h,w,cin,cout", [
    (3, 23, 29, 128, 512),     # layer2's conv3 shape class, 2001 positions: a ragged last 64-row tile
    (2, 14, 14, 256, 1024),    # layer3
    (1, 37, 41, 256, 256),     # two 128-wide column blocks, ragged
    (2, 9, 7, 128, 256),       # fewer row tiles than workgroups: most walk nothing
    (2, 7, 7, 512, 2048),      # layer4 (pw_res2: weights in VGPRs, 16-row tiles)
    (3, 5, 9, 512, 256),       # 135 positions: ragged last 16-row tile, one column block
    (1, 11, 13, 512, 768),     # three column blocks, ragged
])
def test_pw_res_bottleneck_conv3(n, h, w, cin, cout, dt):
    """pw_res (ResNet's conv3 + bn3 + ReLU + identity + ReLU at K = 128 /
    256: weights resident in LDS, input rows and residual blocks streamed by
    global_load_lds; K = 512: pw_res2, weights in VGPRs) into a channel slot of a wider buffer: against PyTorch
    fp32 of the same 16-bit operands within one 16-bit ulp, against the
    convnd_pt route (fac_set_option pw_res = 0) within one ulp, the channels
    around the slot untouched."""
    from fac_fake_amd.ops import ConvLayer
    g = torch.Generator().manual_seed(5 + cin + cout + h)
    x = torch.randn(n, cin, 1, h, w, generator=g).to(T16[dt]).float()
    wt = torch.randn(cout, cin, 1, 1, 1, generator=g) / np.sqrt(cin)
    b = torch.randn(cout, generator=g) * 0.1
    res = torch.randn(n, 1, h, w, cout, generator=g).to(T16[dt])
    layer = ConvLayer(wt, b, 1, 0, dtype=dt, device=DEV)
    xg = x.permute(0, 2, 3, 4, 1).contiguous().to(T16[dt]).to(DEV)
    outs = {}
    try:
        for v in (1, 0):
            _set_knob(b"pw_res", v, dt)
            big = torch.full((n, 1, h, w, cout + 16), 3.0, dtype=T16[dt], device=DEV)
            layer(xg, relu=True, out=big, c_off=8, residual=res.to(DEV), relu2=True)
            torch.cuda.synchronize()
            outs[v] = big.cpu()
    finally:
        _set_knob(b"pw_res", 1, dt)
    conv = F.conv3d(x, wt.to(T16[dt]).float(), b).permute(0, 2, 3, 4, 1)
    ref = F.relu(F.relu(conv) + res.float()).to(T16[dt])
    bc = outs[1]
    u = _ulps(bc[..., 8:8 + cout], ref, dt)
    assert u.max() <= 1.0 and (u > 0).float().mean() <= 0.05, float(u.max())
    assert _ulps(bc, outs[0], dt).max() <= 1.0
    assert torch.all(bc[..., :8] == 3.0) and torch.all(bc[..., 8 + cout:] == 3.0)


@pytest.mark.parametrize("dt", ["bf16", "fp16"])
@pytest.mark.parametrize("case", [
    # (n, h, cin3, hx, cin_ds, stride_ds, cout): ResNet-50 bottleneck conv3 + downsample
    (2, 56, 64, 56, 64, 1, 256),      # layer1 (two K steps: one per GEMM; pw_res DUAL)
    (3, 13, 64, 13, 64, 1, 256),      # layer1 shape class, 507 positions: a ragged last 128-row tile
    (2, 28, 128, 56, 256, 2, 512),    # layer2: strided downsample gather
    (2, 7, 512, 14, 1024, 2, 2048),   # layer4
    (3, 13, 128, 26, 256, 2, 128),    # ragged last row tile, one column block
])
def test_conv_dual_vs_torch_fp32(case, dt):
    """fac_conv_nd_dual (convnd_pt DUAL): relu(relu(conv3(h) + b3) + ds(x) +
    b_ds) in one launch vs PyTorch fp32 of the same 16-bit operands, within one
    16-bit ulp (the downsample sum stays fp32 until the final rounding)."""
    from fac_fake_amd.ops import ConvLayer, conv_dual
    n, hh, c3, hx, cds, sds, cout = case
    g = torch.Generator().manual_seed(7 + cout + hh)
    h = torch.randn(n, c3, 1, hh, hh, generator=g).to(T16[dt]).float()
    x = torch.randn(n, cds, 1, hx, hx, generator=g).to(T16[dt]).float()
    w3 = torch.randn(cout, c3, 1, 1, 1, generator=g) / np.sqrt(c3)
    wd = torch.randn(cout, cds, 1, 1, 1, generator=g) / np.sqrt(cds)
    b3 = torch.randn(cout, generator=g) * 0.1
    bd = torch.randn(cout, generator=g) * 0.1
    l3 = ConvLayer(w3, b3, 1, 0, dtype=dt, device=DEV)
    ld = ConvLayer(wd, bd, (1, sds, sds), 0, dtype=dt, device=DEV)
    hg = h.permute(0, 2, 3, 4, 1).contiguous().to(T16[dt]).to(DEV)
    xg = x.permute(0, 2, 3, 4, 1).contiguous().to(T16[dt]).to(DEV)
    out = conv_dual(l3, hg, ld, xg)
    torch.cuda.synchronize()
    a = F.relu(F.conv3d(h, w3.to(T16[dt]).float(), b3))
    r = F.conv3d(x, wd.to(T16[dt]).float(), bd, stride=(1, sds, sds))
    ref = F.relu(a + r).permute(0, 2, 3, 4, 1).to(T16[dt])
    u = _ulps(out.cpu(), ref, dt)
    assert u.max() <= 1.0 and (u > 0).float().mean() <= 0.05


@pytest.mark.parametrize("dt", ["bf16", "fp16"])
@pytest.mark.parametrize("case", [
    # (n, h, cout, c3, cds): a bottleneck's end, conv3 c3 -> cout at h^2 and
    # the downsample cds -> cout at stride 2 over the (2h)^2 block input
    (2, 28, 512, 128, 256),   # layer2's real shape (pw_dual2, two 256-column blocks)
    (1, 9, 256, 128, 256),    # 81 positions: ragged last 32-row tile, one column block
    (5, 11, 768, 128, 256),   # 605 positions, three column blocks, ragged last tile
    (1, 5, 128, 128, 256),    # cout not a multiple of 256: stays on convnd_pt (both arms)
    (2, 14, 1024, 256, 512),  # layer3's real shape (32 columns per wave, 16-row tiles)
    (1, 9, 256, 256, 512),    # 81 positions: ragged last 16-row tile
    (3, 5, 512, 256, 512),    # 75 positions over two column blocks
])
def test_pw_dual2_layer2(case, dt):
    """fac_conv_nd_dual's layer2 / layer3 route (ops.hip pw_dual2: both
    weight blocks in VGPRs, the strided downsample rows gathered by
    global_load_lds) vs PyTorch fp32 of the same operands, and vs the generic
    convnd_pt DUAL route (fac_set_option "pw_res" 2) within one 16-bit ulp."""
    from fac_fake_amd.ops import ConvLayer, conv_dual
    n, hh, cout, c3, cds = case
    g = torch.Generator().manual_seed(11 + cout + hh)
    h = torch.randn(n, c3, 1, hh, hh, generator=g).to(T16[dt]).float()
    x = torch.randn(n, cds, 1, 2 * hh, 2 * hh, generator=g).to(T16[dt]).float()
    w3 = torch.randn(cout, c3, 1, 1, 1, generator=g) / np.sqrt(c3)
    wd = torch.randn(cout, cds, 1, 1, 1, generator=g) / np.sqrt(cds)
    b3 = torch.randn(cout, generator=g) * 0.1
    bd = torch.randn(cout, generator=g) * 0.1
    l3 = ConvLayer(w3, b3, 1, 0, dtype=dt, device=DEV)
    ld = ConvLayer(wd, bd, (1, 2, 2), 0, dtype=dt, device=DEV)
    hg = h.permute(0, 2, 3, 4, 1).contiguous().to(T16[dt]).to(DEV)
    xg = x.permute(0, 2, 3, 4, 1).contiguous().to(T16[dt]).to(DEV)
    outs = {}
    try:
        for v in (1, 2):
            _set_knob(b"pw_res", v, dt)
            outs[v] = conv_dual(l3, hg, ld, xg)
            torch.cuda.synchronize()
            outs[v] = outs[v].cpu()
    finally:
        _set_knob(b"pw_res", 1, dt)
    a = F.relu(F.conv3d(h, w3.to(T16[dt]).float(), b3))
    r = F.conv3d(x, wd.to(T16[dt]).float(), bd, stride=(1, 2, 2))
    ref = F.relu(a + r).permute(0, 2, 3, 4, 1).to(T16[dt])
    u = _ulps(outs[1], ref, dt)
    assert u.max() <= 1.0 and (u > 0).float().mean() <= 0.05, float(u.max())
    assert _ulps(outs[1], outs[2], dt).max() <= 1.0


@pytest.mark.parametrize("dt", ["bf16", "fp16"])
def test_conv_nd_residual_concat_and_f32(dt):
    """Bottleneck epilogue relu(relu(conv + b) + res) into a channel slot of a
    wider buffer; and fp32 output of a 1-channel conv (S3D's final layer)."""
    from fac_fake_amd.ops import ConvLayer
    g = torch.Generator().manual_seed(7)
    n, h, w, cin, cout = 2, 11, 13, 32, 48
    x = torch.randn(n, cin, 1, h, w, generator=g).to(T16[dt]).float()
    wt = torch.randn(cout, cin, 1, 3, 3, generator=g) / 17.0
    b = torch.randn(cout, generator=g) * 0.1
    res = torch.randn(n, 1, h, w, cout, generator=g).to(T16[dt])
    layer = ConvLayer(wt, b, 1, (0, 1, 1), dtype=dt, device=DEV)
    big = torch.zeros(n, 1, h, w, 128, dtype=T16[dt], device=DEV)
    xg = x.permute(0, 2, 3, 4, 1).contiguous().to(T16[dt]).to(DEV)
    layer(xg, relu=True, out=big[..., :], c_off=40, residual=None)
    out2 = layer(xg, relu=True, residual=res.to(DEV), relu2=True)
    torch.cuda.synchronize()
    conv = F.conv3d(x, wt.to(T16[dt]).float(), b, padding=(0, 1, 1)).permute(0, 2, 3, 4, 1)
    ref1 = F.relu(conv).to(T16[dt])
    ref2 = F.relu(F.relu(conv) + res.float()).to(T16[dt])
    bc = big.cpu()
    assert _ulps(bc[..., 40:40 + cout], ref1, dt).max() <= 1.0
    assert bc[..., :40].abs().max() == 0 and bc[..., 40 + cout:].abs().max() == 0
    assert _ulps(out2.cpu(), ref2, dt).max() <= 1.0
    one = ConvLayer(wt[:1], b[:1], 1, (0, 1, 1), dtype=dt, device=DEV)
    y = one(xg, relu=False, out_f32=True)
    torch.cuda.synchronize()
    ref = F.conv3d(x, wt[:1].to(T16[dt]).float(), b[:1], padding=(0, 1, 1)).permute(0, 2, 3, 4, 1)
    assert y.dtype == torch.float32 and torch.allclose(y.cpu(), ref, rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("dt", ["bf16", "fp16"])
def test_pool_nd(dt):
    from fac_fake_amd.ops import pool
    g = torch.Generator().manual_seed(3)
    x = torch.randn(2, 24, 5, 17, 17, generator=g).to(T16[dt])
    xg = x.permute(0, 2, 3, 4, 1).contiguous().to(DEV)
    ym = pool(xg, (1, 3, 3), (1, 2, 2), (0, 1, 1), "max")   # pool_max_win (compile-time windows)
    y3 = pool(xg, (3, 3, 3), (2, 2, 2), (1, 1, 1), "max")
    y2 = pool(xg, 2, 2, 0, "max")
    y5 = pool(xg, (1, 5, 3), (1, 3, 2), (0, 2, 1), "max")   # pool_nd (no compile-time window)
    ya = pool(xg, (2, 17, 17), (2, 17, 17), 0, "avg")
    torch.cuda.synchronize()
    rm = F.max_pool3d(x.float(), (1, 3, 3), (1, 2, 2), (0, 1, 1)).permute(0, 2, 3, 4, 1)
    r3 = F.max_pool3d(x.float(), 3, 2, 1).permute(0, 2, 3, 4, 1)
    r2 = F.max_pool3d(x.float(), 2, 2).permute(0, 2, 3, 4, 1)
    r5 = F.max_pool3d(x.float(), (1, 5, 3), (1, 3, 2), (0, 2, 1)).permute(0, 2, 3, 4, 1)
    ra = F.avg_pool3d(x.float(), (2, 17, 17)).permute(0, 2, 3, 4, 1)
    assert torch.equal(ym.cpu().float(), rm) and torch.equal(y3.cpu().float(), r3)
    assert torch.equal(y2.cpu().float(), r2) and torch.equal(y5.cpu().float(), r5)
    assert _ulps(ya.cpu(), ra.to(T16[dt]), dt).max() <= 1.0


@pytest.mark.parametrize("dt", ["bf16", "fp16"])
@pytest.mark.parametrize("d", [1, 2, 5])
def test_max_pool_3x3x3_s1(dt, d):
    """The one-pass sliding-window kernel for MaxPool3d(3, 1, 1) (S3D's
    Inception branch3): bit-exact vs torch, also into a channel slot."""
    from fac_fake_amd.ops import max_pool_sep, pool
    g = torch.Generator().manual_seed(5 + d)
    x = torch.randn(3, 40, d, 9, 13, generator=g).to(T16[dt])
    xg = x.permute(0, 2, 3, 4, 1).contiguous().to(DEV)
    y = max_pool_sep(xg, 3, 1, 1)
    big = torch.zeros(3, d, 9, 13, 64, dtype=T16[dt], device=DEV)
    pool(xg, 3, 1, 1, "max", out=big, c_off=16)
    torch.cuda.synchronize()
    r = F.max_pool3d(x.float(), 3, 1, 1).permute(0, 2, 3, 4, 1)
    assert torch.equal(y.cpu().float(), r)
    bc = big.cpu().float()
    assert torch.equal(bc[..., 16:56], r) and bc[..., :16].abs().max() == 0 and bc[..., 56:].abs().max() == 0


@pytest.mark.parametrize("dt", ["bf16", "fp16"])
@pytest.mark.parametrize("d,h,roll", [(4, 7, 1), (1, 7, 1), (5, 3, 1), (6, 9, 4), (5, 7, 2), (4, 7, 0)])
def test_max_pool_3x3x3_s1_roll(dt, d, h, roll):
    """maxpool3_roll (MaxPool3d(3, 1, 1) on 7-wide maps, rolled along the row
    and the frames; pool_roll 1 = every frame in one thread, k = k frames per
    thread, 0 = maxpool3_s1): bit-exact vs torch, into a channel slot, for
    maps shorter and taller than wide and frame counts not divisible by k."""
    import ctypes
    from fac_fake_amd import _lib
    from fac_fake_amd.ops import pool
    lib = _lib.load()
    hd = ctypes.c_void_p()
    _lib.check(lib.fac_create(0, _lib.DTYPES[dt], ctypes.byref(hd)), None, "fac_create")
    g = torch.Generator().manual_seed(9 + d + h)
    x = torch.randn(3, 48, d, h, 7, generator=g).to(T16[dt])
    xg = x.permute(0, 2, 3, 4, 1).contiguous().to(DEV)
    big = torch.zeros(3, d, h, 7, 64, dtype=T16[dt], device=DEV)
    try:
        _lib.check(lib.fac_set_option(hd, b"pool_roll", roll), hd, "fac_set_option")
        pool(xg, 3, 1, 1, "max", out=big, c_off=8)
        torch.cuda.synchronize()
    finally:
        lib.fac_set_option(hd, b"pool_roll", 1)
        lib.fac_destroy(hd)
    r = F.max_pool3d(x.float(), 3, 1, 1).permute(0, 2, 3, 4, 1)
    bc = big.cpu().float()
    assert torch.equal(bc[..., 8:56], r) and bc[..., :8].abs().max() == 0 and bc[..., 56:].abs().max() == 0


@pytest.mark.parametrize("dt", ["bf16", "fp16"])
@pytest.mark.parametrize("d,c", [(1, 64), (2, 128), (5, 192), (8, 64)])
def test_max_pool_3x3x3_s1_lds14(dt, d, c):
    """maxpool3_lds14 (MaxPool3d(3, 1, 1) on 14x14 maps: one workgroup per
    (clip, 64-channel slice), frames through a -inf-bordered LDS image, the
    frame window rolled in registers): bit-exact vs torch into a channel slot
    of a wider tensor, for 1..8 frames and 1..3 channel slices."""
    from fac_fake_amd.ops import pool
    g = torch.Generator().manual_seed(21 + d + c)
    x = torch.randn(3, c, d, 14, 14, generator=g).to(T16[dt])
    xg = x.permute(0, 2, 3, 4, 1).contiguous().to(DEV)
    big = torch.zeros(3, d, 14, 14, c + 16, dtype=T16[dt], device=DEV)
    pool(xg, 3, 1, 1, "max", out=big, c_off=8)
    torch.cuda.synchronize()
    r = F.max_pool3d(x.float(), 3, 1, 1).permute(0, 2, 3, 4, 1)
    bc = big.cpu().float()
    assert torch.equal(bc[..., 8:8 + c], r) and bc[..., :8].abs().max() == 0 and bc[..., 8 + c:].abs().max() == 0


@pytest.mark.parametrize("dt", ["bf16", "fp16"])
@pytest.mark.parametrize("n,d,h,cin,cout,c_off", [
    (2, 8, 14, 192, 32, 8),      # Mixed_3b branch3 at 112^2 clips (one 32-channel block)
    (3, 8, 14, 256, 64, 0),      # Mixed_3c
    (3, 5, 14, 64, 64, 16),      # 4b at the harness's 20 x 224^2 clips: 5 frames
    (3, 4, 7, 480, 64, 16),      # 4b at 112^2: K chunks of 64 with a half-empty last one, 4 frames per unit
    (2, 4, 7, 528, 128, 0),      # 4f: one 128-column block, a quarter-full last chunk
    (2, 4, 7, 64, 256, 8),       # two 128-column blocks
    (2, 2, 7, 512, 64, 8),       # two frames per unit
    (2, 5, 7, 64, 96, 0),        # one frame per unit, three 32-channel blocks
    (3, 2, 3, 832, 128, 0),      # 5b / 5c at 112^2: 3 x 3 maps
    (2, 3, 3, 64, 32, 8),
])
def test_conv_maxpool3s1_fused(n, d, h, cin, cout, c_off, dt):
    """FAC_CONV_MAXPOOL3S1 (ops.hip maxpool3_pw): S3D's Inception branch3,
    MaxPool3d(3, 1, 1) then a 1x1x1 conv + bias + ReLU in one launch, into a
    channel slot of a wider tensor.  Against PyTorch fp32 of the same 16-bit
    operands (the pool is exact in 16 bits) within one 16-bit ulp, against
    fac_pool_nd + the conv's own kernel within one ulp, and the neighbouring
    channels untouched.  Inputs of both signs (the bf16 max runs on int16
    keys), units that do not fill the last XCD range."""
    from fac_fake_amd.ops import ConvLayer, max_pool_sep
    g = torch.Generator().manual_seed(31 + d + h + cin + cout)
    x = torch.randn(n, cin, d, h, h, generator=g).to(T16[dt]).float()
    wt = torch.randn(cout, cin, 1, 1, 1, generator=g) / np.sqrt(cin)
    b = torch.randn(cout, generator=g) * 0.1
    layer = ConvLayer(wt, b, 1, 0, dtype=dt, device=DEV)
    layer.MAXPOOL3S1_MAPS = (14, 7, 3)   # the ABI's maps (the S3D drop-in fuses 14 and 7)
    xg = x.permute(0, 2, 3, 4, 1).contiguous().to(T16[dt]).to(DEV)
    assert layer.maxpool3s1_ok(xg)
    big = torch.zeros(n, d, h, h, cout + 24, dtype=T16[dt], device=DEV)
    layer(xg, relu=True, out=big, c_off=c_off, maxpool3s1=True)
    unf = layer(max_pool_sep(xg, 3, 1, 1), relu=True)
    torch.cuda.synchronize()
    pooled = F.max_pool3d(x, 3, 1, 1)
    ref = F.relu(F.conv3d(pooled, wt.to(T16[dt]).float(), b)).permute(0, 2, 3, 4, 1).to(T16[dt])
    bc = big.cpu()
    got = bc[..., c_off:c_off + cout]
    u = _ulps(got, ref, dt)
    assert u.max() <= 1.0 and (u > 0).float().mean() <= 0.05, float(u.max())
    assert _ulps(got, unf.cpu(), dt).max() <= 1.0
    assert bc[..., :c_off].abs().max() == 0 if c_off else True
    assert bc[..., c_off + cout:].abs().max() == 0


@pytest.mark.parametrize("dt", ["bf16", "fp16"])
@pytest.mark.parametrize("n,d,h,c_off", [(2, 8, 56, 0), (3, 2, 30, 8), (1, 3, 9, 16)])
def test_conv_prepool3s2_fused(n, d, h, c_off, dt):
    """FAC_CONV_PREPOOL3S2 (ops.hip maxpool2s_pw): S3D's base.1 + base.2,
    MaxPool3d((1,3,3), (1,2,2), (0,1,1)) then a 1x1x1 64 -> 64 conv + bias +
    ReLU in one launch, on 56-wide maps of 56 / 30 / 9 rows (the last band of
    4 pooled rows partial for 30 and 9), into a channel slot: against PyTorch
    fp32 of the same 16-bit operands within one 16-bit ulp, against
    fac_pool_nd + the conv's own kernel within one ulp, the neighbouring
    channels untouched.  Inputs of both signs."""
    from fac_fake_amd.ops import ConvLayer, pool
    g = torch.Generator().manual_seed(41 + d + h)
    x = torch.randn(n, 64, d, h, 56, generator=g).to(T16[dt]).float()
    wt = torch.randn(64, 64, 1, 1, 1, generator=g) / 8.0
    b = torch.randn(64, generator=g) * 0.1
    layer = ConvLayer(wt, b, 1, 0, dtype=dt, device=DEV)
    xg = x.permute(0, 2, 3, 4, 1).contiguous().to(T16[dt]).to(DEV)
    assert layer.prepool3s2_ok(xg)
    ho = (h - 1) // 2 + 1
    big = torch.full((n, d, ho, 28, 64 + 24), 5.0, dtype=T16[dt], device=DEV)
    layer(xg, relu=True, out=big, c_off=c_off, prepool3s2=True)
    unf = layer(pool(xg, (1, 3, 3), (1, 2, 2), (0, 1, 1), "max"), relu=True)
    torch.cuda.synchronize()
    pooled = F.max_pool3d(x, (1, 3, 3), (1, 2, 2), (0, 1, 1))
    ref = F.relu(F.conv3d(pooled, wt.to(T16[dt]).float(), b)).permute(0, 2, 3, 4, 1).to(T16[dt])
    bc = big.cpu()
    got = bc[..., c_off:c_off + 64]
    u = _ulps(got, ref, dt)
    assert u.max() <= 1.0 and (u > 0).float().mean() <= 0.05, float(u.max())
    assert _ulps(got, unf.cpu(), dt).max() <= 1.0
    assert torch.all(bc[..., :c_off] == 5.0) and torch.all(bc[..., c_off + 64:] == 5.0)


@pytest.mark.parametrize("dt", ["bf16", "fp16"])
@pytest.mark.parametrize("h,w,pb,pa", [(30, 26, 2, 1), (224, 224, 2, 1), (18, 16, 0, 0)])
def test_pack_input_s2d_u8_cells(h, w, pb, pa, dt):
    """fac_pack_input_s2d on uint8 NHWC images (ResNet-50's conv1 input,
    /255 + ImageNet normalisation): every 16-channel cell is the
    normalised 2x2 pixel block (pixel (dy, dx) in channels 4(2dy+dx) + c,
    channel 3 of each pixel zero), the border cells zero — bit-equal to the
    same arithmetic in fp32 rounded once."""
    from fac_fake_amd.ops import TORCH16, pack_input_s2d
    g = torch.Generator().manual_seed(h + w)
    img = torch.randint(0, 256, (3, h, w, 3), generator=g, dtype=torch.uint8)
    mean, std = (0.485, 0.456, 0.406), (0.229, 0.224, 0.225)
    out = pack_input_s2d(img.to(DEV), dtype=dt, u8=True, div=255.0, mean=mean, std=std, pad_before=pb,
                         pad_after=pa)
    torch.cuda.synchronize()
    ho, wo = h // 2 + pb + pa, w // 2 + pb + pa
    ref = torch.zeros(3, 1, ho, wo, 16)
    x = (img.float() / 255.0 - torch.tensor(mean)) / torch.tensor(std)
    for dy in range(2):
        for dx in range(2):
            blk = x[:, dy:2 * (h // 2):2, dx:2 * (w // 2):2, :]          # [3, h/2, w/2, 3]
            ref[:, 0, pb:pb + h // 2, pb:pb + w // 2, 4 * (2 * dy + dx):4 * (2 * dy + dx) + 3] = blk
    assert tuple(out.shape) == (3, 1, ho, wo, 16)
    assert torch.equal(out.cpu().float(), ref.to(TORCH16[dt]).float())


def test_kan_linear_vs_reference(golden):
    from fac_fake_amd.ops import KANLinearLayer
    g = golden("resvitkan_golden.npz")
    sd = {k: torch.from_numpy(np.asarray(v)) for k, v in make_resvitkan_state_dict(0).items()}
    p = "kan_head.3.layers.0"
    layer = KANLinearLayer(sd[p + ".grid"], sd[p + ".base_weight"], sd[p + ".spline_weight"],
                           sd[p + ".spline_scaler"], DEV)
    y = layer(torch.from_numpy(g["kan_x"]).to(DEV))
    torch.cuda.synchronize()
    assert np.abs(y.cpu().numpy() - g["kan_y"]).max() <= 1e-5


@pytest.fixture(scope="module")
def rvk():
    from fac_fake_amd.resvitkan import ResVitKan
    sd = {k: torch.from_numpy(np.asarray(v)) for k, v in make_resvitkan_state_dict(0).items()}
    out = {}
    for dt in ("fp16", "bf16"):
        m = ResVitKan(dtype=dt)
        m.load_state_dict(sd)
        out[dt] = m
    return out


@pytest.mark.parametrize("dt", ["fp16", "bf16"])
def test_resvitkan_matches_reference(rvk, golden, dt, tol16):
    from oracle.cvit_torch import normalize_u8
    tol = tol16(dt, "resvitkan_golden.npz")
    g = golden("resvitkan_golden.npz")
    crops = make_crops(4, seed=int(g["crop_seed"]))
    m = rvk[dt]
    lg_u8 = m.forward_u8(torch.from_numpy(crops).to(DEV))
    lg_f32 = m(normalize_u8(crops).to(DEV))
    torch.cuda.synchronize()
    p_ref = 1 / (1 + np.exp(-g["logits"].astype(np.float64)))
    for lg in (lg_u8, lg_f32):
        p = 1 / (1 + np.exp(-lg.cpu().numpy().astype(np.float64)))
        assert np.abs(p - p_ref).max() <= tol


@pytest.mark.parametrize("dt", ["fp16", "bf16"])
def test_resvitkan_every_block_matches_reference(rvk, golden, dt):
    """8 crops: the per-channel means of the max-pool output, of EVERY Bottleneck
    (layer1..layer4, downsample and residual included) and of bn2 against the
    reference module's (tests/golden/resvitkan_golden_stages.npz), within 2x
    that stage's emulated 16-bit envelope; probabilities fp16 within 1e-3,
    bf16 within 2x its emulated envelope."""
    g = golden("resvitkan_golden_stages.npz")
    n = int(g["n_crops"])
    x = torch.from_numpy(make_crops(n, seed=int(g["crop_seed"]))).to(DEV)
    m = rvk[dt]
    taps = m.stage_outputs(x)
    torch.cuda.synchronize()
    assert len(taps) == 18
    env = g[f"env_{dt}"]
    for i, t in enumerate(taps):
        got = t.float().reshape(n, -1, t.shape[-1]).mean(1).double().cpu().numpy()
        ref = g[f"mean_{i}"].astype(np.float64)
        assert got.shape == ref.shape, (i, got.shape, ref.shape)
        err = float(np.abs(got - ref).max() / np.sqrt((ref ** 2).mean()))
        assert err <= 2 * env[i] + 1e-4, (i, err, env[i])
    lg, pr = m.forward_u8(x, pos_index=torch.arange(n, dtype=torch.int32), return_probs=True)
    p_ref = 1 / (1 + np.exp(-g["logits"].astype(np.float64)))
    bar = 1e-3 if dt == "fp16" else 2 * float(g[f"env_prob_{dt}"])
    assert np.abs(pr.double().cpu().numpy() - p_ref).max() <= bar


def test_resvitkan_features_match_emulation(rvk, golden):
    """The ResNet-50 stem alone vs the oracle's emulation of the same 16-bit
    rounding points (fp16): relative error of the [B,7,7,512] features."""
    from oracle import resvitkan_torch as O
    from oracle.cvit_torch import normalize_u8, to_torch_sd
    from fac_fake_amd.ops import pack_input_s2d
    g = golden("resvitkan_golden.npz")
    x = normalize_u8(make_crops(2, seed=int(g["crop_seed"])))
    m = rvk["fp16"]
    f = m.features16(pack_input_s2d(x.to(DEV), dtype="fp16", u8=False))
    torch.cuda.synchronize()
    ref = O.resnet50_emulated(to_torch_sd(make_resvitkan_state_dict(0)), x, "fp16").permute(0, 2, 3, 1)
    err = (f.cpu().float().reshape(ref.shape) - ref).abs().max() / ref.abs().max()
    assert err <= 5e-3


def test_resvitkan_graph_replay_matches_eager(rvk):
    m = rvk["bf16"]
    crops = torch.from_numpy(make_crops(8, seed=5)).to(DEV)
    eager = m.forward_u8(crops).clone()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        m.forward_u8(crops)
        torch.cuda.synchronize()
        gr = torch.cuda.CUDAGraph()
        with torch.cuda.graph(gr, stream=s):
            out = m.forward_u8(crops)
    gr.replay()
    torch.cuda.synchronize()
    assert torch.equal(out, eager)


# ---------------------------------------------------------------- S3D (config 4)
@pytest.fixture(scope="module")
def s3d_models():
    from fac_fake_amd.s3d import S3D
    from fac_fake_amd.weights import make_s3d_state_dict
    out = {}
    for srm in ("no", "yes"):
        sd = {k: torch.from_numpy(np.asarray(v)) for k, v in make_s3d_state_dict(0, 1, srm == "yes").items()}
        for dt in ("fp16", "bf16"):
            m = S3D(1, srm, dtype=dt)
            m.load_state_dict(sd)
            out[(srm, dt)] = m
    return out


@pytest.mark.parametrize("srm", ["no", "yes"])
@pytest.mark.parametrize("dt", ["fp16", "bf16"])
def test_s3d_matches_reference(s3d_models, golden, srm, dt, tol16):
    """Per-logit sigmoid of 2 raw 16x112x112 clips vs the reference module (golden)."""
    tol = tol16(dt, f"s3d_golden.npz:{srm}")
    from fac_fake_amd.weights import s3d_clips
    g = golden("s3d_golden.npz")
    x = torch.from_numpy(s3d_clips(2, 16, 112, seed=int(g["clip_seed"]))).to(DEV)
    lg, pr = s3d_models[(srm, dt)](x, return_probs=True)
    lg8 = s3d_models[(srm, dt)](x.to(torch.uint8))   # decoded-frame input: the same integer values
    torch.cuda.synchronize()
    p_ref = 1 / (1 + np.exp(-g[f"logits_{srm}"].astype(np.float64)))
    assert lg.shape == (2, 1)
    assert np.abs(pr.cpu().numpy() - p_ref).max() <= tol
    assert torch.equal(lg8, lg)


@pytest.mark.parametrize("srm", ["no", "yes"])
@pytest.mark.parametrize("dt", ["fp16", "bf16"])
def test_s3d_reference_harness_shape(s3d_models, golden, srm, dt):
    """The reference harness's clip shape (S3D-test.py:130-190: 200 frames,
    every 10th kept -> 20; model.py:344-354 profiles 20 x 224 x 224): 2 raw
    content-varied clips through the drop-in vs the reference module
    (tests/golden/s3d_golden_20x224.npz).  fp16 within the 1e-3 bar, bf16
    within 1.25x the oracle's emulated bf16 envelope at this shape (plus
    the accumulation-order allowance, conftest.ORDER_NOISE)."""
    from fac_fake_amd.weights import s3d_clips_varied
    g = golden("s3d_golden_20x224.npz")
    x = torch.from_numpy(s3d_clips_varied(2, int(g["frames"]), int(g["size"]), seed=int(g["clip_seed"]))).to(DEV)
    lg, pr = s3d_models[(srm, dt)](x, return_probs=True)
    torch.cuda.synchronize()
    p_ref = 1 / (1 + np.exp(-g[f"logits_{srm}"].astype(np.float64)))
    from conftest import bf16_gate
    tol = 1e-3 if dt == "fp16" else bf16_gate(float(g[f"env_prob_{srm}_bf16"]))
    assert lg.shape == (2, 1)
    assert np.abs(pr.cpu().numpy() - p_ref).max() <= tol, (np.abs(pr.cpu().numpy() - p_ref).max(), tol)


def _rel_to_rms(got, ref):
    return float(np.abs(got - ref).max() / (np.sqrt((ref.astype(np.float64) ** 2).mean()) + 1e-30))


@pytest.mark.parametrize("srm", ["no", "yes"])
@pytest.mark.parametrize("dt", ["fp16", "bf16"])
def test_s3d_every_block_matches_reference(s3d_models, golden, srm, dt):
    """8 content-varied clips: the per-channel means of EVERY base[i] output
    (stem convs, pools, each Mixed_* block's four concatenated branches) against
    the reference module's (tests/golden/s3d_golden_blocks.npz), within 2x the
    16-bit rounding envelope of that layer (the oracle's emulation of the HIP
    path's rounding points vs fp32, stored with the fixture).  A wrong branch,
    channel slot or stride moves a layer's channel means by O(rms), far past
    the 0.1-6 % envelopes.  Probabilities: fp16 within 1e-3 (the north-star
    bar), bf16 within 2x its emulated envelope."""
    from fac_fake_amd.weights import s3d_clips_varied
    g = golden("s3d_golden_blocks.npz")
    x = torch.from_numpy(s3d_clips_varied(int(g["n_clips"]), 16, 112, int(g["clip_seed"]))).to(DEV)
    m = s3d_models[(srm, dt)]
    taps = m.base_outputs(x)
    torch.cuda.synchronize()
    assert len(taps) == 16
    env = g[f"env_{srm}_{dt}"]
    for i, t in enumerate(taps):
        got = t.float().mean(dim=(1, 2, 3)).double().cpu().numpy()
        ref = g[f"mean_{srm}_{i}"].astype(np.float64)
        assert got.shape == ref.shape, (i, got.shape, ref.shape)
        err = _rel_to_rms(got, ref)
        assert err <= 2 * env[i] + 1e-4, (i, err, env[i])
    lg, pr = m(x, return_probs=True)
    p_ref = 1 / (1 + np.exp(-g[f"logits_{srm}"].astype(np.float64)))
    bar = 1e-3 if dt == "fp16" else 2 * float(g[f"env_prob_{srm}_{dt}"])
    assert np.abs(pr.double().cpu().numpy() - p_ref).max() <= bar


def test_s3d_video_predictions(s3d_models, golden):
    """S3D-test.py's per-video score (sigmoid per row, mean, [0]) for 8 videos of
    one snippet each, in batches of 3 (ragged last batch): the reference's
    probabilities within 1e-3 (fp16) and custom_round's labels."""
    from fac_fake_amd.s3d import custom_round, video_predictions
    from fac_fake_amd.weights import s3d_clips_varied
    g = golden("s3d_golden_blocks.npz")
    x = torch.from_numpy(s3d_clips_varied(int(g["n_clips"]), 16, 112, int(g["clip_seed"]))).to(DEV)
    preds = video_predictions(s3d_models[("no", "fp16")], x, batch=3)
    p_ref = 1 / (1 + np.exp(-g["logits_no"].astype(np.float64)))[:, 0]
    assert len(preds) == 8 and np.abs(np.array(preds) - p_ref).max() <= 1e-3
    assert np.array_equal(custom_round(preds), custom_round(p_ref))


def test_s3d_matches_emulation_tightly(s3d_models, golden):
    """fp16 path vs the oracle's emulation of its rounding points: logits within 2e-3."""
    from oracle import s3d_torch as O
    from fac_fake_amd.weights import make_s3d_state_dict, s3d_clips
    g = golden("s3d_golden.npz")
    x = torch.from_numpy(s3d_clips(2, 16, 112, seed=int(g["clip_seed"])))
    ref = O.forward_emulated(make_s3d_state_dict(0, 1, False), x, False, "fp16")
    lg = s3d_models[("no", "fp16")](x.to(DEV))
    torch.cuda.synchronize()
    assert (lg.cpu() - ref).abs().max() <= 2e-3


@pytest.mark.parametrize("hw", [(128, 128), (96, 160), (112, 56)])
def test_s3d_clip_sizes_outside_the_fused_tiling(s3d_models, hw):
    """base.0's fused s2d conv (fac_conv_s2d4_clip) tiles H % 16,
    W % 56; other clip sizes (the reference takes any, model.py:43) take the
    packed-cell route on the generic conv.  (112, 56) is on the fused route
    at a width the bench never uses.  fp16 vs the oracle's emulation of the
    HIP rounding points (logits within 2e-3, as the 112^2 test) and the fp32
    oracle within the 1e-3 probability bar; a uint8 clip gives the same
    logits as its float copy."""
    from oracle import s3d_torch as O
    from fac_fake_amd.weights import make_s3d_state_dict, s3d_clips_varied
    h, w = hw
    x = torch.from_numpy(s3d_clips_varied(2, 16, max(h, w), seed=7))[..., :h, :w].contiguous()
    sd = make_s3d_state_dict(0, 1, False)
    m = s3d_models[("no", "fp16")]
    lg, pr = m(x.to(DEV), return_probs=True)
    lg8 = m(x.to(torch.uint8).to(DEV))
    torch.cuda.synchronize()
    emu = O.forward_emulated(sd, x, False, "fp16")
    ref = O.forward_fp32(sd, x, False)
    assert lg.shape == (2, 1) and torch.isfinite(lg).all()
    assert (lg.cpu() - emu).abs().max() <= 2e-3, (lg.cpu(), emu)
    assert (pr.cpu().double() - torch.sigmoid(ref.double())).abs().max() <= 1e-3
    assert torch.equal(lg8, lg)


def test_s3d_graph_replay_matches_eager(s3d_models):
    from fac_fake_amd.weights import s3d_clips
    m = s3d_models[("yes", "bf16")]
    x = torch.from_numpy(s3d_clips(3, 16, 112, seed=5)).to(DEV)
    eager = m(x).clone()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        m(x)
        torch.cuda.synchronize()
        gr = torch.cuda.CUDAGraph()
        with torch.cuda.graph(gr, stream=s):
            out = m(x)
    gr.replay()
    torch.cuda.synchronize()
    assert torch.equal(out, eager)


@pytest.mark.parametrize("dt", ["bf16", "fp16"])
@pytest.mark.parametrize("pt_wide,shape", [(32, (2, 4, 7, 7)), (1, (2, 4, 7, 7)), (1, (3, 8, 14, 14))])
def test_conv_split_equals_separate_convs(dt, pt_wide, shape):
    """fac_conv_nd_split over concatenated weights (S3D's merged Inception
    heads) writes exactly what three separate fac_conv_nd launches write:
    on convnd_igemm (the default at this size) and on convnd_pt's column
    segments (nd_pt_wide = 1: any row-tile count; 304 columns = two full
    128-wide blocks and a partial one)."""
    g = torch.Generator().manual_seed(11)
    (n, d, h, w), cin, widths = shape, 480, (192, 96, 16)
    _nd_pt_wide(pt_wide, dt)
    try:
        _split_case(g, n, d, h, w, cin, widths, dt)
    finally:
        _nd_pt_wide(32, dt)


@pytest.mark.parametrize("dt", ["bf16", "fp16"])
@pytest.mark.parametrize("shape,cin,widths", [
    ((3, 8, 14, 14), 192, (64, 96, 16)),     # Mixed_3b's heads: 176 columns = two 128-wide blocks, ragged rows
    ((3, 8, 14, 14), 256, (128, 128, 32)),   # Mixed_3c's heads: 288 = three blocks, the last a quarter full
    ((1, 1, 5, 7), 256, (64, 96, 16)),       # fewer row tiles than workgroups
])
def test_pw_res_split_heads(shape, cin, widths, dt):
    """fac_conv_nd_split at K = 192 / 256 on pw_res PLAIN (S3D's merged
    Inception heads at 14 x 14: weights resident in LDS, input rows streamed):
    each column segment within one 16-bit ulp of its own fac_conv_nd launch
    (other kernels, other summation order) and of PyTorch fp32 on the same
    operands, the rest of the concat buffer untouched."""
    from fac_fake_amd.ops import ConvLayer, conv_split
    g = torch.Generator().manual_seed(13 + cin)
    n, d, h, w = shape
    x = torch.randn(n, d, h, w, cin, generator=g).to(T16[dt])
    ws = [torch.randn(c, cin, 1, 1, 1, generator=g) / np.sqrt(cin) for c in widths]
    bs = [torch.randn(c, generator=g) * 0.1 for c in widths]
    sep = [ConvLayer(wi, bi, 1, 0, dtype=dt, device=DEV) for wi, bi in zip(ws, bs)]
    merged = ConvLayer(torch.cat(ws), torch.cat(bs), 1, 0, dtype=dt, device=DEV)
    xg = x.to(DEV)
    out = torch.zeros(n, d, h, w, 512, dtype=T16[dt], device=DEV)
    h1 = torch.empty(n, d, h, w, widths[1], dtype=T16[dt], device=DEV)
    h2 = torch.empty(n, d, h, w, widths[2], dtype=T16[dt], device=DEV)
    conv_split(merged, xg, (widths[0], widths[0] + widths[1]), out, 0, h1, h2)
    rs = [layer(xg) for layer in sep]
    torch.cuda.synchronize()
    xf = x.float().permute(0, 4, 1, 2, 3)
    got = [out[..., :widths[0]].cpu(), h1.cpu(), h2.cpu()]
    for gi, ri, wi, bi in zip(got, rs, ws, bs):
        ref = F.relu(F.conv3d(xf, wi.to(T16[dt]).float(), bi)).permute(0, 2, 3, 4, 1).to(T16[dt])
        u = _ulps(gi, ref, dt)
        assert u.max() <= 1.0 and (u > 0).float().mean() <= 0.05, float(u.max())
        assert _ulps(gi, ri.cpu(), dt).max() <= 1.0
    assert out[..., widths[0]:].abs().max() == 0


@pytest.mark.parametrize("dt", ["bf16", "fp16"])
@pytest.mark.parametrize("n", [3, 300])
@pytest.mark.parametrize("cin,cmid", [(16, 32), (32, 96)])
def test_sep_tiny_equals_two_launches(n, cin, cmid, dt):
    """fac_sep_tiny / fac_sep_mid (Mixed_3b's / 3c's branch2 SepConv3d, 16 ->
    32 -> 32 / 32 -> 96 -> 96 on 8 x 14 x 14, in one launch with the middle
    map in LDS) into a channel slot, against PyTorch fp32 with the map
    rounded to 16 bits as both routes store it: within two 16-bit ulps of the
    output scale, and no further from it than the two fac_conv_nd launches
    plus one such ulp (a map value one ulp apart from fp32 summation order
    moves an output through the 96 / 288-term temporal sum, so per-element
    ulps of near-zero outputs say nothing); 300 clips make every workgroup
    walk several clips / bands."""
    from fac_fake_amd.ops import ConvLayer, sep_tiny
    g = torch.Generator().manual_seed(61 + n + cin)
    x = torch.randn(n, 8, 14, 14, cin, generator=g).to(T16[dt])
    w1 = torch.randn(cmid, cin, 1, 3, 3, generator=g) / (3.0 * cin ** 0.5)
    b1 = torch.randn(cmid, generator=g) * 0.1
    w2 = torch.randn(cmid, cmid, 3, 1, 1, generator=g) / (1.7 * cmid ** 0.5)
    b2 = torch.randn(cmid, generator=g) * 0.1
    if cmid == 96:   # S3D's padding of Mixed_3c's middle channels to 128 (zero rows / biases, s3d.py m2w)
        s = ConvLayer(torch.cat([w1, w1.new_zeros(32, cin, 1, 3, 3)]), torch.cat([b1, b1.new_zeros(32)]), 1,
                      (0, 1, 1), dtype=dt, device=DEV)
        t = ConvLayer(w2, b2, 1, (1, 0, 0), dtype=dt, device=DEV, cin_pad=128)
    else:
        s = ConvLayer(w1, b1, 1, (0, 1, 1), dtype=dt, device=DEV)
        t = ConvLayer(w2, b2, 1, (1, 0, 0), dtype=dt, device=DEV)
    xg = x.to(DEV)
    big = torch.full((n, 8, 14, 14, cmid + 16), 2.0, dtype=T16[dt], device=DEV)
    sep_tiny(s, t, xg, big, 8)
    two = t(s(xg))
    torch.cuda.synchronize()
    xf = x.float().permute(0, 4, 1, 2, 3)
    mid = F.relu(F.conv3d(xf, w1.to(T16[dt]).float(), b1, padding=(0, 1, 1))).to(T16[dt]).float()
    ref = F.relu(F.conv3d(mid, w2.to(T16[dt]).float(), b2, padding=(1, 0, 0))).permute(0, 2, 3, 4, 1).to(T16[dt])
    bc = big.cpu()
    got = bc[..., 8:8 + cmid]
    scale = ref.float().abs().max()
    ulp = 2.0 ** (torch.floor(torch.log2(scale)) - (7 if dt == "bf16" else 10))
    e1 = (got.float() - ref.float()).abs().max()
    e2 = (two.cpu().float() - ref.float()).abs().max()
    assert e1 <= 2 * ulp and e1 <= e2 + ulp, (float(e1), float(e2), float(ulp))
    assert torch.all(bc[..., :8] == 2.0) and torch.all(bc[..., 8 + cmid:] == 2.0)


def _split_case(g, n, d, h, w, cin, widths, dt):
    from fac_fake_amd.ops import ConvLayer, conv_split
    x = torch.randn(n, d, h, w, cin, generator=g).to(T16[dt]).to(DEV)
    ws = [torch.randn(c, cin, 1, 1, 1, generator=g) / np.sqrt(cin) for c in widths]
    bs = [torch.randn(c, generator=g) * 0.1 for c in widths]
    sep = [ConvLayer(wi, bi, 1, 0, dtype=dt, device=DEV) for wi, bi in zip(ws, bs)]
    merged = ConvLayer(torch.cat(ws), torch.cat(bs), 1, 0, dtype=dt, device=DEV)
    out = torch.zeros(n, d, h, w, 512, dtype=T16[dt], device=DEV)
    h1 = torch.empty(n, d, h, w, widths[1], dtype=T16[dt], device=DEV)
    h2 = torch.empty(n, d, h, w, widths[2], dtype=T16[dt], device=DEV)
    conv_split(merged, x, (widths[0], widths[0] + widths[1]), out, 0, h1, h2)
    r0, r1, r2 = (layer(x) for layer in sep)
    torch.cuda.synchronize()
    assert torch.equal(out[..., :widths[0]], r0) and out[..., widths[0]:].abs().max() == 0
    assert torch.equal(h1, r1) and torch.equal(h2, r2)


@pytest.mark.parametrize("dt", ["fp16", "bf16"])
def test_s3d_base0_fused_equals_two_launches(s3d_models, dt):
    """base.0 (SepConv3d 3->64, k 7, s 2) of a uint8
    16 x 112 x 112 clip batch as one launch (fac_s3d_base0_u8) is
    bit-identical to conv_s2d4_clip_u8 + the temporal conv_tk2, for a batch
    whose units do not divide the persistent grid, and the whole S3D forward
    with it equals the forward without it."""
    from fac_fake_amd import ops
    from fac_fake_amd.weights import s3d_clips
    m = s3d_models[("no", dt)]
    x = torch.from_numpy(s3d_clips(3, 16, 112, seed=77)).to(DEV).to(torch.uint8)
    m._pack(x)
    kind, L = m._layers[0]
    assert kind == "sep_s2d"
    fused = ops.s3d_base0_u8(L[0], L[1], x.contiguous())
    two = L[1](ops.conv_s2d4_clip(L[0], x.contiguous()))
    torch.cuda.synchronize()
    assert fused.shape == two.shape == (3, 8, 56, 56, 64)
    assert torch.equal(fused.view(torch.int16), two.view(torch.int16))
    a = m(x)
    m.fuse_base0 = False
    try:
        b = m(x)
    finally:
        m.fuse_base0 = True
    torch.cuda.synchronize()
    assert torch.equal(a, b)
