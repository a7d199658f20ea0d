"""HIP path vs the oracle and the reference's goldens, through the C ABI.

Tolerances (stated per test):
* fp16 operands: per-frame probabilities within 1e-3 of the fp32 reference
  (the north-star bar), checked against goldens the reference produced.
* bf16 operands: exact bf16 rounding of the operands alone already moves the
  fp32 reference by 1.5e-3 .. 5.3e-3 in probability on these fixtures (the
  oracle's emulation, tests/golden/bf16_envelope.json), so
  end-to-end bf16 is gated at 1.25x that envelope per fixture plus 5e-4
  for the HIP path's fp32 summation order (conftest tol16 / bf16_gate), and
  the kernels themselves are gated
  tightly per kernel: each conv fed the oracle's previous-layer output agrees
  to <= 2 ulp (1-ulp accumulation-order flips on a few % of outputs), the
  tail fed the oracle's stem output agrees within 1e-3 in probability, and
  the whole forward stays inside the oracle's 16-bit rounding envelope.
"""
import numpy as np
import pytest
import torch

from fac_fake_amd.weights import make_crops

pytestmark = pytest.mark.gpu

DEV = "cuda:0"


def _sig(x):
    return 1.0 / (1.0 + np.exp(-np.asarray(x, np.float64)))


@pytest.fixture(scope="module")
def models(sd, built_lib):
    assert torch.cuda.is_available(), "GPU tests need a visible MI355X"
    from fac_fake_amd.cvit import CViT
    out = {}
    for dt in ("fp16", "bf16"):
        m = CViT(dtype=dt)
        m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in sd.items()})
        m.to(DEV)
        m.reserve(256, DEV)
        out[dt] = m
    return out


def _run_u8(m, crops, slots):
    x = torch.from_numpy(crops).to(DEV)
    lg = m.forward_u8(x, pos_index=torch.from_numpy(np.asarray(slots, np.int32)))
    torch.cuda.synchronize()
    return lg.cpu().numpy()


def test_native_library_is_the_one_loaded(models):
    from fac_fake_amd import _lib
    lib = _lib.load()
    assert lib.fac_version().decode().startswith("fac_cvit")
    maps = open("/proc/self/maps").read()
    assert str(_lib.LIB_PATH) in maps


@pytest.mark.parametrize("dt", ["fp16", "bf16"])
def test_c1_single_crop(models, golden, dt, tol16):
    g = golden("golden_c1.npz")
    crops = make_crops(1, seed=1)
    assert int(crops.astype(np.int64).sum()) == int(g["crop_sum"])
    lg = _run_u8(models[dt], crops, [0])
    dp = np.abs(_sig(lg) - g["probs"]).max()
    assert np.isfinite(lg).all()
    assert dp <= tol16(dt, "golden_c1.npz"), (dt, dp, lg, g["logits"])


@pytest.mark.parametrize("dt", ["fp16", "bf16"])
def test_b32_all_slots(models, golden, dt, tol16):
    g = golden("golden_b32.npz")
    crops = make_crops(32, seed=2)
    lg = _run_u8(models[dt], crops, np.arange(32))
    dp = np.abs(_sig(lg) - _sig(g["logits"])).max()
    assert dp <= tol16(dt, "golden_b32.npz"), (dt, dp)


@pytest.mark.parametrize("dt", ["fp16", "bf16"])
def test_b256_config2(models, golden, dt, tol16):
    """Config 2: B=256 crops in one call, slot = j mod 32 (8 reference chunks of 32)."""
    g = golden("golden_b256.npz")
    crops = make_crops(256, seed=3)
    lg = _run_u8(models[dt], crops, np.arange(256) % 32)
    dp = np.abs(_sig(lg) - _sig(g["logits"])).max()
    assert dp <= tol16(dt, "golden_b256.npz"), (dt, dp)


@pytest.mark.parametrize("dt", ["fp16", "bf16"])
def test_real_crops(models, golden, dt, tol16):
    g = golden("golden_real.npz")
    lg = _run_u8(models[dt], g["crops"], [0, 1])
    dp = np.abs(_sig(lg) - _sig(g["logits"])).max()
    assert dp <= tol16(dt, "golden_real.npz"), (dt, dp)


ULP_REL = {"fp16": 2.0 ** -10, "bf16": 2.0 ** -7}  # one unit in the last place, relative


def _ulp_diff(got, ref, dt):
    """|got - ref| in 16-bit ulps of max(|ref|, rms(ref)/2).

    The floor matters for outputs near zero: there the fp32 accumulation-order
    noise (relative to the summed magnitudes, not to the tiny result) exceeds
    a 16-bit ulp of the result.  A wrong tap/channel/pixel is off by O(rms):
    hundreds of these units."""
    floor = 0.5 * float(ref.pow(2).mean().sqrt())
    return ((got - ref).abs() / (ref.abs().clamp_min(floor) * ULP_REL[dt])).max().item()


def _rms_rel(a, b):
    return float((a - b).pow(2).mean().sqrt() / (b.pow(2).mean().sqrt() + 1e-30))


@pytest.mark.parametrize("dt", ["fp16", "bf16"])
def test_conv1_fused_normalize_vs_oracle(models, sd, dt, torch_threads):
    """conv1 with the uint8 -> /255 -> Normalize step fused: bit-exact but for
    accumulation-order rounding flips (at most 1 ulp, on a tiny fraction)."""
    from fac_fake_amd import _lib
    from oracle.cvit_torch import forward_emulated, normalize_u8
    crops = make_crops(2, seed=12)
    _, feats = forward_emulated(sd, normalize_u8(crops), dtype=dt, return_features=True)
    ref = feats[0].permute(0, 2, 3, 1).contiguous()
    lib = _lib.load()
    x = torch.from_numpy(crops).to(DEV)
    out = torch.empty(ref.shape, dtype=torch.float16 if dt == "fp16" else torch.bfloat16, device=DEV)
    _lib.check(lib.fac_debug_features_u8(models[dt]._ctx, x.data_ptr(), 2, 0, out.data_ptr(), None), None, "dbg")
    torch.cuda.synchronize()
    got = out.float().cpu()
    assert float((got != ref).float().mean()) <= 1e-3
    assert _ulp_diff(got, ref, dt) <= 1.01


@pytest.mark.parametrize("dt", ["fp16", "bf16"])
def test_each_conv_kernel_isolated(models, sd, dt, torch_threads):
    """Every stem conv (conv2..conv17, all six kernel instantiations) fed the
    oracle's previous-layer output: BN-fold, ReLU, fused max-pool and the
    16-bit store must agree with the oracle up to 1-ulp accumulation-order
    flips on a small fraction of outputs."""
    from fac_fake_amd import _lib
    from oracle.cvit_torch import conv_block_emulated, forward_emulated, normalize_u8
    crops = make_crops(2, seed=12)
    _, feats = forward_emulated(sd, normalize_u8(crops), dtype=dt, return_features=True)
    lib = _lib.load()
    tdt = torch.float16 if dt == "fp16" else torch.bfloat16
    for layer in range(1, 17):
        inp = feats[layer - 1]
        ref = conv_block_emulated(sd, inp, layer, dt).permute(0, 2, 3, 1).contiguous()
        x = inp.permute(0, 2, 3, 1).contiguous().to(tdt).to(DEV)
        out = torch.empty(ref.shape, dtype=tdt, device=DEV)
        _lib.check(lib.fac_debug_conv(models[dt]._ctx, layer, x.data_ptr(), 2, out.data_ptr(), None), None, "conv")
        torch.cuda.synchronize()
        got = out.float().cpu()
        frac = float((got != ref).float().mean())
        assert frac <= 0.05, (layer, frac)
        assert _ulp_diff(got, ref, dt) <= 2.01, (layer, _ulp_diff(got, ref, dt))


@pytest.mark.parametrize("dt", ["fp16", "bf16"])
def test_fused_stem224_vs_unfused_and_oracle(models, sd, dt, torch_threads):
    """The fused conv1..conv3+pool kernel (stem224.hip) against the same three
    convs run one kernel each, and against the oracle emulation."""
    from fac_fake_amd import _lib
    from oracle.cvit_torch import forward_emulated, normalize_u8
    crops = make_crops(3, seed=17)
    _, feats = forward_emulated(sd, normalize_u8(crops), dtype=dt, return_features=True)
    ref = feats[2].permute(0, 2, 3, 1).contiguous()
    lib = _lib.load()
    m = models[dt]
    x = torch.from_numpy(crops).to(DEV)
    tdt = torch.float16 if dt == "fp16" else torch.bfloat16
    outs = {}
    for fuse in (1, 0):
        _lib.check(lib.fac_set_option(m._ctx, b"fuse_stem224", fuse), m._ctx, "opt")
        o = torch.empty(ref.shape, dtype=tdt, device=DEV)
        _lib.check(lib.fac_debug_features_u8(m._ctx, x.data_ptr(), 3, 2, o.data_ptr(), None), m._ctx, "dbg")
        torch.cuda.synchronize()
        outs[fuse] = o.float().cpu()
    _lib.check(lib.fac_set_option(m._ctx, b"fuse_stem224", 1), m._ctx, "opt")
    fused, unfused = outs[1], outs[0]
    # the fused kernel accumulates bias-first: a different, equally valid fp32
    # summation order, so a few % of 16-bit roundings may flip by one ulp
    assert float((fused != unfused).float().mean()) <= 0.02
    assert _ulp_diff(fused, unfused, dt) <= 2.01
    assert float((fused != ref).float().mean()) <= 0.05
    assert _ulp_diff(fused, ref, dt) <= 4.01


@pytest.mark.parametrize("dt", ["fp16", "bf16"])
def test_tail_isolated(models, sd, dt, torch_threads):
    """Patch embedding + 6 transformer layers + head from the oracle's stem
    output: within the 16-bit rounding envelope of the fp32 tail."""
    from fac_fake_amd import _lib
    from oracle.cvit_torch import forward_emulated, normalize_u8, tail_emulated, tail_fp32
    crops = make_crops(8, seed=11)
    slots = np.array([0, 5, 31, 7, 7, 12, 30, 1])
    _, feats = forward_emulated(sd, normalize_u8(crops), dtype=dt, return_features=True)
    stem = feats[16]
    em = tail_emulated(sd, stem, slots, dt)
    fp = tail_fp32(sd, stem, slots)
    lib = _lib.load()
    x = stem.permute(0, 2, 3, 1).contiguous().to(torch.float16 if dt == "fp16" else torch.bfloat16).to(DEV)
    p = torch.from_numpy(slots.astype(np.int32)).to(DEV)
    out = torch.empty(8, 2, device=DEV)
    _lib.check(lib.fac_debug_tail(models[dt]._ctx, x.data_ptr(), 8, p.data_ptr(), out.data_ptr(), None), None, "tail")
    torch.cuda.synchronize()
    got = out.cpu()
    print(dt, "tail gpu-emu", float((got - em).abs().max()), "emu-fp32", float((em - fp).abs().max()),
          "gpu-fp32", float((got - fp).abs().max()))
    assert _rms_rel(got, fp) <= 1.5 * _rms_rel(em, fp) + 1e-4
    # bf16 rounding-order noise alone is ~1e-3 here (emulation vs fp32: ~2e-3)
    assert np.abs(_sig(got.numpy()) - _sig(em.numpy())).max() <= (1e-3 if dt == "fp16" else 2.5e-3)


@pytest.mark.parametrize("dt", ["fp16", "bf16"])
def test_error_envelope_end_to_end(models, sd, dt, torch_threads):
    """Whole forward: the HIP path's distance from fp32 is what exact 16-bit
    rounding at its rounding points gives (oracle emulation), not more."""
    from oracle.cvit_torch import forward_emulated, forward_fp32, normalize_u8
    crops = make_crops(8, seed=11)
    slots = np.array([0, 5, 31, 7, 7, 12, 30, 1])
    x = normalize_u8(crops)
    em = forward_emulated(sd, x, pos_index=slots, dtype=dt)
    fp = forward_fp32(sd, x, pos_index=slots)
    got = torch.from_numpy(_run_u8(models[dt], crops, slots))
    assert _rms_rel(got, fp) <= 1.6 * _rms_rel(em, fp) + 1e-4, (_rms_rel(got, fp), _rms_rel(em, fp))


def test_nchw_f32_matches_u8(models):
    """forward(img) on reference-normalised fp32 == forward_u8 (normalisation fused in conv1)."""
    from oracle.cvit_torch import normalize_u8
    m = models["fp16"]
    crops = make_crops(4, seed=13)
    a = _run_u8(m, crops, np.arange(4))
    img = normalize_u8(crops).to(DEV)
    b = m(img).detach().cpu().numpy()
    assert np.array_equal(a, b)


def test_pos_slot_permutation_is_exact(models):
    m = models["fp16"]
    crops = make_crops(16, seed=14)
    slots = np.arange(16) * 2 % 32
    a = _run_u8(m, crops, slots)
    perm = np.random.default_rng(0).permutation(16)
    b = _run_u8(m, crops[perm], slots[perm])
    assert np.array_equal(a[perm], b)


def test_ragged_batches_and_edge_sizes(models, golden):
    g = golden("golden_b32.npz")
    m = models["fp16"]
    crops = make_crops(32, seed=2)
    for B in (1, 2, 3, 17, 31):
        lg = _run_u8(m, crops[:B], np.arange(B))
        assert np.abs(_sig(lg) - _sig(g["logits"][:B])).max() <= 1e-3, B
    # an empty batch gives empty outputs, as the reference's forward does
    e = m.forward_u8(torch.from_numpy(crops[:0]).to(DEV), return_probs=True)
    assert tuple(e[0].shape) == (0, 2) and tuple(e[1].shape) == (0, 2)
    assert tuple(m(torch.zeros(0, 3, 224, 224, device=DEV)).shape) == (0, 2)


def test_reference_forward_contract(models):
    m = models["fp16"]
    with pytest.raises(RuntimeError):
        m(torch.zeros(33, 3, 224, 224, device=DEV))     # pos_embedding[0:33] fails in the reference
    with pytest.raises(RuntimeError):
        m(torch.zeros(1, 3, 224, 224))                   # no CPU fallback
    out = m(torch.zeros(2, 3, 224, 224, device=DEV))
    assert out.shape == (2, 2) and out.dtype == torch.float32


def test_mask_argument_matches_the_reference(models):
    """forward(img, mask): all-True masks change nothing, any False gives NaN
    logits for every crop, B not in {1, 8} raises (tests/golden/mask_semantics.json)."""
    from oracle.cvit_torch import normalize_u8
    m = models["fp16"]
    img = normalize_u8(make_crops(8, seed=21)).to(DEV)
    base = m(img).cpu()
    keep = torch.ones(8, 1, dtype=torch.bool)
    assert torch.equal(m(img, mask=keep).cpu(), base)
    drop = keep.clone()
    drop[3, 0] = False
    assert torch.isnan(m(img, mask=drop)).all()
    with pytest.raises(RuntimeError):
        m(img[:2], mask=keep[:2])


def test_out_of_range_pos_index_is_an_error_at_the_c_abi(models):
    """SURVEY §8b error convention: a pos_index outside [0,32) cannot be
    reported by the kernel that reads it, so the device clamps it and raises
    a host-visible flag; the context's next forward returns FAC_ERR_ARG (and
    enqueues nothing), and fac_check_device_errors reports it after a sync."""
    import ctypes
    from fac_fake_amd import _lib
    lib = _lib.load()
    m = models["fp16"]
    ctx = m._ctx
    x = torch.from_numpy(make_crops(4, seed=19)).to(DEV)
    lg = torch.empty(4, 2, device=DEV)
    good = torch.tensor([0, 1, 2, 3], dtype=torch.int32, device=DEV)
    bad = torch.tensor([0, 1, 40, 3], dtype=torch.int32, device=DEV)
    st = torch.cuda.current_stream().cuda_stream
    # eager forwards (the small-batch graph replay bakes in its capture's
    # number; covered below)
    m.set_option("graph_max_b", 0)
    try:
        assert lib.fac_forward_nhwc_u8(ctx, x.data_ptr(), 4, bad.data_ptr(), lg.data_ptr(), None, st) == 0
        torch.cuda.synchronize()
        rc = lib.fac_forward_nhwc_u8(ctx, x.data_ptr(), 4, good.data_ptr(), lg.data_ptr(), None, st)
        msg = lib.fac_last_error(ctx)
        # the error names the offending forward: launch #n, the next #n+1
        import re
        got = re.search(rb"encoder launch #(\d+) of this context \(the next is #(\d+)", msg)
        assert rc == -1 and b"pos_index" in msg and got and int(got.group(2)) == int(got.group(1)) + 1, msg
        assert lib.fac_forward_nhwc_u8(ctx, x.data_ptr(), 4, good.data_ptr(), lg.data_ptr(), None, st) == 0  # cleared
        assert lib.fac_forward_nhwc_u8(ctx, x.data_ptr(), 4, bad.data_ptr(), lg.data_ptr(), None, st) == 0
        flags = ctypes.c_int()
        assert lib.fac_check_device_errors(ctx, ctypes.byref(flags)) == 0 and flags.value == int(got.group(1)) + 2
        assert lib.fac_check_device_errors(ctx, ctypes.byref(flags)) == 0 and flags.value == 0
        assert lib.fac_forward_nhwc_u8(ctx, x.data_ptr(), 4, good.data_ptr(), lg.data_ptr(), None, st) == 0
        torch.cuda.synchronize()
    finally:
        m.set_option("graph_max_b", 32)
    # the graph replay path raises the same flag and the next call is refused
    assert lib.fac_forward_nhwc_u8(ctx, x.data_ptr(), 4, bad.data_ptr(), lg.data_ptr(), None, st) == 0
    torch.cuda.synchronize()
    assert lib.fac_forward_nhwc_u8(ctx, x.data_ptr(), 4, good.data_ptr(), lg.data_ptr(), None, st) == -1
    assert lib.fac_forward_nhwc_u8(ctx, x.data_ptr(), 4, good.data_ptr(), lg.data_ptr(), None, st) == 0
    torch.cuda.synchronize()


def test_chunked_video_prediction(models, golden):
    """predict()'s chunking on 40 crops ([0:32] then [32:40]) and the video score."""
    from fac_fake_amd.prediction import predict_crops
    g = golden("golden_chunks.npz")
    crops = make_crops(40, seed=4)
    score = predict_crops(models["fp16"], torch.from_numpy(crops))
    assert abs(score - float(g["score"])) <= 1e-3


def test_device_video_score(models, golden):
    from fac_fake_amd import _lib
    lib = _lib.load()
    for row in golden("golden_postproc.json"):
        n = row["n"]
        lg = torch.tensor(np.asarray(row["logits"], np.float32).reshape(-1, 2), device=DEV)
        out = torch.empty((), dtype=torch.float32, device=DEV)
        _lib.check(lib.fac_video_score(lg.data_ptr() if n else None, n, out.data_ptr(),
                                       torch.cuda.current_stream().cuda_stream), None, "video_score")
        assert abs(out.item() - row["score"]) <= 1e-6, n


def test_graph_capture_replay_matches_eager(models):
    from fac_fake_amd import _lib
    m = models["fp16"]
    lib = _lib.load()
    crops = torch.from_numpy(make_crops(64, seed=15)).to(DEV)
    pidx = (torch.arange(64, device=DEV) % 32).to(torch.int32)
    eager = m.forward_u8(crops, pos_index=pidx.cpu()).clone()
    out = torch.empty(64, 2, device=DEV)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            _lib.check(lib.fac_forward_nhwc_u8(m._ctx, crops.data_ptr(), 64, pidx.data_ptr(), out.data_ptr(), None,
                                               s.cuda_stream), m._ctx, "capture")
    g.replay()
    torch.cuda.synchronize()
    assert torch.equal(out, eager)


def test_stem_chunking_is_bit_exact(models):
    """Running conv1..conv9 in sub-batches (Infinity-Cache-sized stem chunks)
    changes nothing: same kernels per crop, so logits and features are identical."""
    from fac_fake_amd import _lib
    lib = _lib.load()
    m = models["fp16"]
    crops = make_crops(100, seed=18)
    slots = np.arange(100) % 32
    base = _run_u8(m, crops, slots)
    x = torch.from_numpy(crops[:40]).to(DEV)
    feats = {}
    for chunk in (0, 48, 17):
        _lib.check(lib.fac_set_option(m._ctx, b"stem_chunk", chunk), m._ctx, "opt")
        if chunk:
            assert np.array_equal(_run_u8(m, crops, slots), base), chunk
        f = torch.empty(40, 56, 56, 64, dtype=torch.float16, device=DEV)
        _lib.check(lib.fac_debug_features_u8(m._ctx, x.data_ptr(), 40, 5, f.data_ptr(), None), m._ctx, "dbg")
        torch.cuda.synchronize()
        feats[chunk] = f.cpu()
    _lib.check(lib.fac_set_option(m._ctx, b"stem_chunk", 0), m._ctx, "opt")
    assert torch.equal(feats[0], feats[48]) and torch.equal(feats[0], feats[17])


def test_large_batch_properties(models):
    """B=512 (beyond the goldens): finite, and bit-identical to scoring the same crops as a B=64 batch."""
    m = models["fp16"]
    crops = make_crops(512, seed=16)
    slots = np.arange(512) % 32
    big = _run_u8(m, crops, slots)
    assert np.isfinite(big).all()
    small = _run_u8(m, crops[448:], slots[448:])
    assert np.array_equal(big[448:], small)     # a crop's logits do not depend on its batch


@pytest.mark.parametrize("variant", [0, 1, 2, 3, 4, 5, 6])
@pytest.mark.parametrize("dt", ["fp16", "bf16"])
def test_gemm_variants_vs_torch_fp32(models, dt, variant):
    """Every GEMM tile variant and epilogue vs a torch fp32 matmul of the same
    16-bit operands (fp32 accumulation: only the summation order differs, so
    |err| <= 1e-5 * sum|a*w| per output).  M = 200 exercises the row clamp
    (M not a multiple of the tile), K = 1024 / splits 4 the partial slabs."""
    m = models[dt]
    tdt = torch.float16 if dt == "fp16" else torch.bfloat16
    g = torch.Generator(device="cpu").manual_seed(7 + variant)
    M, N, K = 200, 384, 1024
    a = (torch.randn(M, K, generator=g) * 0.5).to(tdt).to(DEV)
    w = (torch.randn(N, K, generator=g) * 0.05).to(tdt).to(DEV)
    bias = torch.randn(N, generator=g).to(DEV)
    ref = a.float() @ w.float().t()
    bound = 1e-5 * (a.float().abs() @ w.float().abs().t()) + 1e-6

    def run(epi, out, splits=1):
        m.debug_gemm(epi, a, w, bias, out, splits=splits, variant=variant)
        torch.cuda.synchronize()
        return out

    o = run(0, torch.empty(M, N, device=DEV))
    assert ((o - (ref + bias)).abs() <= bound).all()
    o = run(1, torch.empty(M, N, device=DEV))
    assert ((o - torch.relu(ref + bias)).abs() <= bound).all()
    base = torch.randn(M, N, generator=g).to(DEV)
    o = run(3, base.clone())
    assert ((o - (base + ref + bias)).abs() <= bound + 1e-6 * base.abs()).all()
    slabs = run(4, torch.empty(4, M, N, device=DEV), splits=4)
    assert ((slabs.sum(0) - ref).abs() <= bound).all()
    ref4 = torch.stack([a[:, i * 256:(i + 1) * 256].float() @ w[:, i * 256:(i + 1) * 256].float().t()
                        for i in range(4)])
    assert ((slabs - ref4).abs() <= bound).all()
    # 16-bit outputs: within one rounding of the fp32 result
    o = run(5, torch.empty(M, N, dtype=tdt, device=DEV)).float()
    r = (ref + bias).to(tdt).float()
    ulp = torch.finfo(tdt).eps * r.abs().clamp_min(torch.finfo(tdt).tiny)
    assert ((o - r).abs() <= ulp + bound).all()
    o = run(2, torch.empty(M, N, dtype=tdt, device=DEV)).float()
    r = torch.nn.functional.gelu(ref + bias).to(tdt).float()
    ulp = torch.finfo(tdt).eps * r.abs().clamp_min(1e-3)
    assert ((o - r).abs() <= ulp + 2 * bound).all()


def test_pipelined_forward_matches_synchronous(models):
    """fac_forward_nhwc_u8_pipelined (batch k's encoder on the context's
    stream, overlapping batch k+1's conv stack) gives bit-identical logits,
    probabilities and video scores to the synchronous forward, over 5
    back-to-back batches of different sizes and a synchronous forward issued
    in the middle of the pipeline."""
    from fac_fake_amd import _lib
    lib = _lib.load()
    m = models["bf16"]
    ctx = m._ctx
    sizes = [64, 64, 17, 64, 40]
    batches = [torch.from_numpy(make_crops(n, seed=100 + i)).to(DEV) for i, n in enumerate(sizes)]
    slots = [(torch.arange(n, device=DEV) % 32).to(torch.int32) for n in sizes]
    ref = []
    for x, p in zip(batches, slots):
        ref.append(m.forward_u8(x, pos_index=p.cpu()).cpu())
    s = torch.cuda.Stream(DEV)
    outs = [torch.full((n, 2), float("nan"), device=DEV) for n in sizes]
    probs = [torch.full((n, 2), float("nan"), device=DEV) for n in sizes]
    scores = [torch.full((), float("nan"), device=DEV) for _ in sizes]
    with torch.cuda.stream(s):
        for i, (x, p) in enumerate(zip(batches, slots)):
            _lib.check(lib.fac_forward_nhwc_u8_pipelined(ctx, x.data_ptr(), sizes[i], p.data_ptr(),
                                                         outs[i].data_ptr(), probs[i].data_ptr(),
                                                         scores[i].data_ptr(), s.cuda_stream), ctx, "pipelined")
            if i == 2:  # a synchronous forward in the middle orders itself after the pending tails
                mid = m.forward_u8(batches[0], pos_index=slots[0].cpu())
        _lib.check(lib.fac_pipeline_join(ctx, 0, s.cuda_stream), ctx, "join")
    torch.cuda.synchronize()
    assert torch.equal(mid.cpu(), ref[0])
    for i in range(len(sizes)):
        assert torch.equal(outs[i].cpu(), ref[i]), i
        assert torch.equal(probs[i].cpu(), torch.sigmoid(ref[i]).float()) or \
            torch.allclose(probs[i].cpu(), torch.sigmoid(ref[i]), rtol=0, atol=1e-6)
        sc = torch.empty((), device=DEV)
        _lib.check(lib.fac_video_score(outs[i].data_ptr(), sizes[i], sc.data_ptr(),
                                       torch.cuda.current_stream().cuda_stream), None, "video_score")
        torch.cuda.synchronize()
        assert torch.equal(scores[i].cpu(), sc.cpu()), i


def test_forward_u8_pipelined_chunks_match(models):
    """CViT.forward_u8_pipelined (equal chunks through the pipelined C ABI,
    chunk k's encoder beside chunk k+1's conv stack) == one forward_u8 call,
    bit for bit, for 2, 5 and 1 chunk(s) and both dtypes."""
    crops = torch.from_numpy(make_crops(300, seed=31)).to(DEV)
    slots = torch.from_numpy((np.arange(300) % 32).astype(np.int32))
    for dt in ("bf16", "fp16"):
        m = models[dt]
        ref = m.forward_u8(crops, pos_index=slots).cpu()
        for chunk in (160, 64, 300):
            got = m.forward_u8_pipelined(crops, slots, chunk=chunk).cpu()
            assert torch.equal(got, ref), (dt, chunk)


def test_crop_resize_kernel_matches_oracle():
    """fac_crop_resize_u8 (crop + INTER_AREA + BGR->RGB) is bit-identical to
    oracle/video.py on downscales (odd and even sizes; exact-integer area
    weights), the 224 identity, boxes under 224 px on one or both axes (cv2's
    bilinear-with-area-coefficients branch: enlargements, mixed
    shrink/enlarge, integer factors, 1-px and 223-px boxes), boxes clipped by
    the frame, empty boxes and out-of-range frame indices."""
    from fac_fake_amd.video import crop_faces
    from oracle import video as ov
    rng = np.random.default_rng(11)
    frames = rng.integers(0, 256, (5, 720, 1280, 3), dtype=np.uint8)
    boxes = np.array([[0, 10, 20, 234, 244], [1, 100, 50, 551, 501], [2, 0, 0, 333, 257], [3, 1000, 400, 1280, 720],
                      [4, 37, 41, 137, 141], [0, 1200, 600, 1500, 900], [1, -30, -40, 270, 260],
                      [2, 5, 5, 5, 300], [9, 0, 0, 300, 300], [4, 640, 0, 641, 720], [3, 3, 7, 1279, 719],
                      [0, 0, 0, 300, 150], [1, 50, 60, 200, 500], [2, 10, 10, 122, 122], [3, 7, 9, 8, 10],
                      [4, 100, 100, 323, 323], [0, 500, 300, 724, 524], [1, 0, 0, 224, 223], [2, 17, 3, 49, 35],
                      [3, 900, 100, 1077, 290]],
                     np.int32)
    got = crop_faces(torch.from_numpy(frames).to(DEV), boxes).cpu().numpy()
    want = ov.crop_batch(frames, boxes)
    assert np.array_equal(got, want)


@pytest.mark.parametrize("mode", ["reference", "dense"])
def test_video_driver_matches_drop_in(models, mode):
    """Config 3 at its stated size on one GPU (BASELINE.json configs[2]: one
    300-frame 1080x1920 video): predict_video's logits are bit-identical to
    the drop-in CViT scoring the oracle's crops with the reference's slots,
    and the score is the reference scoring rule applied to them."""
    from fac_fake_amd.prediction import chunk_slots, dense_slots, pre_process_prediction, pred_sig
    from fac_fake_amd.video import predict_video, reference_boxes, synthetic_video
    from oracle import video as ov
    m = models["bf16"]
    frames, boxes = synthetic_video(300, 1080, 1920, seed=3, device=DEV)
    score, logits = predict_video(m, frames, boxes, mode=mode, return_logits=True)
    sel = reference_boxes(boxes, 300) if mode == "reference" else boxes
    slots = chunk_slots(len(sel)) if mode == "reference" else dense_slots(len(sel))
    crops = torch.from_numpy(ov.crop_batch(frames.cpu().numpy(), sel)).to(DEV)
    ref = m.forward_u8(crops, pos_index=torch.from_numpy(slots)).cpu()
    assert len(sel) == (29 if mode == "reference" else 300)
    assert torch.equal(logits.cpu(), ref)
    # the score is computed on the device (fac_video_score): the reference's
    # rule, up to the sigmoid's last-bit rounding
    assert abs(score - float(pre_process_prediction(pred_sig(ref)))) <= 1e-6


def test_multi_video_batching_matches_per_video(models):
    """predict_videos (config 3's reference workload, cvit_prediction.py:73-83:
    <= 29 crops per video, slots 0..n-1 each) scores many videos' crops in
    shared forwards and reduces them with one segmented score launch: every
    score and every logit is bit-identical to predict_video on that video
    alone, for videos with 0, 1, 2, 3 and 29 crops, host and device frames,
    and batches that split videos across forwards."""
    from fac_fake_amd.video import predict_video, predict_videos, synthetic_video
    m = models["bf16"]
    vids = []
    for i, (n, faces) in enumerate(((300, 1), (40, 1), (10, 1), (20, 1), (30, 1), (120, 3), (7, 1), (60, 2))):
        frames, boxes = synthetic_video(n, 270, 480, seed=11 + i, device=DEV, faces_per_frame=faces, box_min=40,
                                        box_span=200)
        if i == 6:
            boxes = boxes[:0]
        vids.append((frames, boxes))
    want, want_lg = zip(*[predict_video(m, f, b, mode="reference", return_logits=True) for f, b in vids])
    counts = [0 if lg is None else lg.shape[0] for lg in want_lg]
    assert {0, 1, 2, 3, 29} <= set(counts), counts
    ref_lg = torch.cat([lg for lg in want_lg if lg is not None]).cpu()
    for batch, host in ((256, False), (32, False), (7, True)):
        src = [(f.cpu().numpy(), b) if host else (f, b) for f, b in vids]
        got, lg = predict_videos(m, src, batch=batch, device=DEV, return_logits=True)
        assert got == list(want), (batch, got, want)
        assert torch.equal(lg.cpu(), ref_lg), batch


@pytest.mark.parametrize("mode", ["reference", "dense"])
def test_host_frames_upload_only_what_is_cropped(models, mode):
    """A host video (numpy) gives the same score and logits as the same
    video resident on the device: predict_video then uploads only the frames
    its (this rank's) crops come from."""
    from fac_fake_amd.video import predict_video, synthetic_video
    m = models["bf16"]
    frames, boxes = synthetic_video(120, 360, 640, seed=21, device=DEV, faces_per_frame=2)
    s_dev, lg_dev = predict_video(m, frames, boxes, mode=mode, return_logits=True)
    s_host, lg_host = predict_video(m, frames.cpu().numpy(), boxes, mode=mode, return_logits=True)
    assert s_dev == s_host and torch.equal(lg_dev.cpu(), lg_host.cpu())


@pytest.mark.parametrize("cin,cout,pool", [(128, 256, 0), (256, 256, 1), (96, 192, 0), (160, 128, 1), (32, 128, 0)])
@pytest.mark.parametrize("dt", ["bf16", "fp16"])
def test_conv_db_tile_vs_torch_fp32(models, cin, cout, pool, dt):
    """The 28x28 3x3 convs run on conv3x3_db (weight fragments straight into
    registers, register-staged halo, one barrier per 32-channel chunk; its
    LDS-weight-ring twin lost twice and was removed in round 5): every 28^2
    column tile (BN 256 / 192 / 128: CViT, S3D, ResNet), odd and even chunk
    counts, a single chunk, ragged batch, and the fused 2x2 max-pool, against
    torch's fp32 conv of the same 16-bit operands (two 16-bit ulps)."""
    from fac_fake_amd import _lib
    from fac_fake_amd.ops import TORCH16, _zero256
    lib = _lib.load()
    g = torch.Generator().manual_seed(cin + cout + pool)
    n = 5
    x = torch.randn(n, 28, 28, cin, generator=g).relu().to(TORCH16[dt]).to(DEV)
    w = (torch.randn(cout, cin, 3, 3, generator=g) / np.sqrt(9 * cin)).contiguous()
    b = (torch.randn(cout, generator=g) * 0.1).to(DEV)
    ne = lib.fac_conv3x3_packed_elems(28, cin, cout)
    pk = torch.empty(ne, dtype=torch.int16)
    _lib.check(lib.fac_conv3x3_pack(_lib.DTYPES[dt], 28, cin, cout, w.data_ptr(), pk.data_ptr()), None, "pack")
    pk = pk.to(DEV)
    ho = 14 if pool else 28
    outs = []
    for _ in range(2):   # and run to run: bit-identical
        y = torch.empty(n, ho, ho, cout, dtype=TORCH16[dt], device=DEV)
        _lib.check(lib.fac_conv3x3(_lib.DTYPES[dt], x.data_ptr(), pk.data_ptr(), b.data_ptr(), y.data_ptr(), n, 28,
                                   cin, cout, pool, 1, _zero256(x.device).data_ptr(),
                                   torch.cuda.current_stream().cuda_stream), None, "fac_conv3x3")
        outs.append(y)
    torch.cuda.synchronize()
    assert torch.equal(outs[0].view(torch.int16), outs[1].view(torch.int16))
    ref = torch.nn.functional.conv2d(x.cpu().float().permute(0, 3, 1, 2), w.to(TORCH16[dt]).float(), b.cpu(),
                                     padding=1).relu()
    if pool:
        ref = torch.nn.functional.max_pool2d(ref, 2)
    ref = ref.permute(0, 2, 3, 1)
    got = outs[0].cpu().float()
    assert torch.allclose(got, ref, rtol=2 * ULP_REL[dt], atol=1e-2), float((got - ref).abs().max())


def test_stem_event_timing(models):
    """Option stem_events (the bench's roofline source): fac_stem_event_ms
    reports one timed launch per pipelined forward, then resets."""
    import ctypes
    from fac_fake_amd import _lib
    lib = _lib.load()
    m = models["bf16"]
    ctx = m._ctx
    x = torch.from_numpy(make_crops(64, seed=5)).to(DEV)
    p = (torch.arange(64, device=DEV) % 32).to(torch.int32)
    lg = torch.empty(64, 2, device=DEV)
    s = torch.cuda.Stream(DEV)
    m.set_option("stem_events", 1)
    try:
        with torch.cuda.stream(s):
            for _ in range(3):
                _lib.check(lib.fac_forward_nhwc_u8_pipelined(ctx, x.data_ptr(), 64, p.data_ptr(), lg.data_ptr(), None,
                                                             None, s.cuda_stream), ctx, "pipelined")
            _lib.check(lib.fac_pipeline_join(ctx, 0, s.cuda_stream), ctx, "join")
        avg, n = ctypes.c_float(), ctypes.c_int()
        _lib.check(lib.fac_stem_event_ms(ctx, ctypes.byref(avg), ctypes.byref(n)), ctx, "stem_event_ms")
        assert n.value == 3 and 0.0 < avg.value < 100.0, (n.value, avg.value)
        _lib.check(lib.fac_stem_event_ms(ctx, ctypes.byref(avg), ctypes.byref(n)), ctx, "stem_event_ms")
        assert n.value == 0
    finally:
        m.set_option("stem_events", 0)
    torch.cuda.synchronize()


@pytest.mark.parametrize("dt", ["fp16", "bf16"])
def test_small_batch_graph_replay_is_bit_identical(models, dt):
    """forwards of B <= 32 crops (the reference's one-video
    call, cvit_prediction.py:224-229) replay a hipGraph captured per (B,
    input kind, probs).  Logits and probabilities are bit-identical to the
    eager forward (option graph_max_b = 0), for uint8 and fp32 NCHW input,
    interleaved batch sizes (graph cache hits and misses), explicit slots,
    and after new weights are loaded (the graphs are dropped and recaptured)."""
    from oracle.cvit_torch import normalize_u8
    m = models[dt]
    cases = [(1, 3), (29, 4), (7, 5), (29, 6), (32, 7), (1, 8)]
    got = []
    for B, seed in cases:
        u8 = make_crops(B, seed=seed)
        x = torch.from_numpy(u8).to(DEV)
        pidx = torch.from_numpy((np.arange(B) * 7 % 32).astype(np.int32))
        lg, pr = m.forward_u8(x, return_probs=True)
        lg2 = m.forward_u8(x, pos_index=pidx)
        lg3 = m(normalize_u8(u8).to(DEV)) if B <= 8 else None
        got.append((lg.clone(), pr.clone(), lg2.clone(), None if lg3 is None else lg3.clone()))
    m.set_option("graph_max_b", 0)
    try:
        for (B, seed), g in zip(cases, got):
            u8 = make_crops(B, seed=seed)
            x = torch.from_numpy(u8).to(DEV)
            pidx = torch.from_numpy((np.arange(B) * 7 % 32).astype(np.int32))
            lg, pr = m.forward_u8(x, return_probs=True)
            assert torch.equal(g[0], lg) and torch.equal(g[1], pr), B
            assert torch.equal(g[2], m.forward_u8(x, pos_index=pidx)), B
            if g[3] is not None:
                assert torch.equal(g[3], m(normalize_u8(u8).to(DEV))), B
    finally:
        m.set_option("graph_max_b", 32)
    torch.cuda.synchronize()


def test_small_batch_graph_follows_new_weights(sd):
    """Loading a different state_dict drops the captured graphs: the replay
    then matches the eager forward on the new weights."""
    from fac_fake_amd.cvit import CViT
    from fac_fake_amd.weights import make_state_dict
    m = CViT(dtype="fp16")
    m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in sd.items()})
    x = torch.from_numpy(make_crops(5, seed=9)).to(DEV)
    a = m.forward_u8(x).clone()
    m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in make_state_dict(1).items()})
    b = m.forward_u8(x).clone()
    m.set_option("graph_max_b", 0)
    c = m.forward_u8(x)
    torch.cuda.synchronize()
    assert not torch.equal(a, b) and torch.equal(b, c)
    m._release()


def test_weights_changed_in_place_or_swapped_are_used(sd):
    """The forwards launch on the uploaded weights and then check the
    parameters' versions and storages: a parameter changed in place, or
    replaced by a new tensor, after the last upload is re-uploaded and the
    forward re-run, so every result matches a model built on the new
    weights (graph and eager batch sizes)."""
    from fac_fake_amd.cvit import CViT
    sdt = {k: torch.from_numpy(np.asarray(v)) for k, v in sd.items()}
    m = CViT(dtype="fp16")
    m.load_state_dict(sdt)
    for B in (5, 40):
        x = torch.from_numpy(make_crops(B, seed=10 + B)).to(DEV)
        p = (torch.arange(B) % 32).to(torch.int32).to(DEV)
        a = m.forward_u8(x, pos_index=p).clone()
        a2 = m.forward_u8(x, pos_index=p).clone()     # same buffers: the direct-graph path for B = 5
        h2 = getattr(m.mlp_head, "2")
        with torch.no_grad():
            h2.weight.mul_(1.5)
        b = m.forward_u8(x, pos_index=p).clone()
        h2.bias = torch.nn.Parameter(h2.bias.detach() + 0.25)
        c = m.forward_u8(x, pos_index=p).clone()
        ref = CViT(dtype="fp16")
        ref.load_state_dict(m.state_dict())
        rc = ref.forward_u8(x, pos_index=p)
        torch.cuda.synchronize()
        assert torch.equal(a, a2) and not torch.equal(a, b) and not torch.equal(b, c) and torch.equal(c, rc), B
        ref._release()
        m.load_state_dict(sdt)
    m._release()


def test_forwards_on_two_streams_are_ordered(models):
    """calls on one context from different streams share its
    workspace; the C ABI makes each forward wait for the previous one on the
    device.  Two streams, no host sync between the calls, eager (B = 40) and
    graph (B = 20) paths: every result equals the same call made alone."""
    m = models["fp16"]
    xs = [torch.from_numpy(make_crops(n, seed=30 + n)).to(DEV) for n in (40, 20, 40, 20)]
    pos = [(torch.arange(x.shape[0]) % 32).to(torch.int32) for x in xs]   # host slots: no device sync
    alone = []
    for x, p in zip(xs, pos):
        alone.append(m.forward_u8(x, pos_index=p).clone())
    torch.cuda.synchronize()
    streams = [torch.cuda.Stream(DEV), torch.cuda.Stream(DEV)]
    outs = []
    for i, (x, p) in enumerate(zip(xs, pos)):
        s = streams[i & 1]
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            outs.append(m.forward_u8(x, pos_index=p))
    torch.cuda.synchronize()
    for a, b in zip(alone, outs):
        assert torch.equal(a, b)


def test_gemm_tile_variants_are_bit_identical(models):
    """Every GEMM tile (wide 64/32 x 128 and the narrow few-row 64x32 / 32x64
    tiles) sums each output's K in the same order: bit-identical outputs, so
    switching tiles by row count never changes a crop's logits."""
    m = models["fp16"]
    g = torch.Generator(device="cpu").manual_seed(5)
    M, N, K = 58, 3072, 1024
    a = (torch.randn(M, K, generator=g) * 0.5).to(torch.float16).to(DEV)
    w = (torch.randn(N, K, generator=g) * 0.05).to(torch.float16).to(DEV)
    bias = torch.randn(N, generator=g).to(DEV)
    outs = []
    for v in range(7):
        o = torch.empty(M, N, device=DEV)
        m.debug_gemm(0, a, w, bias, o, splits=1, variant=v)
        s = torch.empty(4, M, N, device=DEV)
        m.debug_gemm(4, a, w, bias, s, splits=4, variant=v)
        outs.append((o, s))
    torch.cuda.synchronize()
    for o, s in outs[1:]:
        assert torch.equal(o, outs[0][0]) and torch.equal(s, outs[0][1])


@pytest.mark.parametrize("dt", ["fp16", "bf16"])
def test_few_crop_forward_equals_full_batch(models, dt):
    """The reference's one-video call (29 crops) takes the few-row GEMM tiles
    and the half-width 28^2 / 14^2 conv blocks (fill the CUs at small B); its
    logits are bit-identical to the same crops scored inside a 256-crop batch
    (the wide tiles), and to the same call with both switched off."""
    m = models[dt]
    crops = make_crops(256, seed=77)
    pidx = (np.arange(256) % 32).astype(np.int32)
    big = _run_u8(m, crops, pidx)
    sel = slice(64, 93)
    small = _run_u8(m, crops[sel], pidx[sel])
    assert np.array_equal(big[sel], small)
    m.set_option("conv_small", 0)
    m.set_option("gemm_small", -1)
    try:
        off = _run_u8(m, crops[sel], pidx[sel])
    finally:
        m.set_option("conv_small", 1)
        m.set_option("gemm_small", 5)
    assert np.array_equal(off, small)


@pytest.mark.parametrize("B", [3, 29])
def test_ring9_conv_is_bit_identical(models, B):
    """Option conv_ring9 (the few-crop 14^2 / 28^2 convs with 9-slice weight
    rings) only changes when weight slices are fetched: conv11's, conv13's,
    conv14's and conv17's outputs and the logits are bit-identical to the
    3-slice rings."""
    from fac_fake_amd import _lib
    lib = _lib.load()
    m = models["fp16"]
    x = torch.from_numpy(make_crops(B, seed=69)).to(DEV)
    pidx = (torch.arange(B) % 32).to(torch.int32)
    outs = {}
    try:
        for v in (0, 1, 2, 4, 7):
            m.set_option("conv_ring9", v)
            feats = []
            for layer, shape in ((10, (B, 28, 28, 256)), (12, (B, 14, 14, 256)), (13, (B, 14, 14, 512)),
                                 (16, (B, 7, 7, 512))):
                f = torch.empty(*shape, dtype=torch.float16, device=DEV)
                _lib.check(lib.fac_debug_features_u8(m._ctx, x.data_ptr(), B, layer, f.data_ptr(), None), m._ctx, "dbg")
                feats.append(f.view(torch.int16).cpu())
            lg = m.forward_u8(x, pos_index=pidx)
            torch.cuda.synchronize()
            outs[v] = (feats, lg.cpu())
    finally:
        m.set_option("conv_ring9", 6)
    for v in (1, 2, 4, 7):
        for a, b in zip(outs[0][0], outs[v][0]):
            assert torch.equal(a, b), v
        assert torch.equal(outs[0][1], outs[v][1]), v


@pytest.mark.parametrize("B", [5, 16])
def test_conv_small14_blocks_are_bit_identical(models, B):
    """Option conv_small14 (the few-crop 14^2 convs on 32-channel blocks while
    they fit one workgroup per CU: twice the workgroups of the 64-channel
    ones) only changes which workgroup computes which channels: conv14-17's
    outputs and the logits are bit-identical to the 64-channel blocks."""
    from fac_fake_amd import _lib
    lib = _lib.load()
    m = models["fp16"]
    x = torch.from_numpy(make_crops(B, seed=83)).to(DEV)
    pidx = (torch.arange(B) % 32).to(torch.int32)
    outs = {}
    try:
        for v in (0, 1):
            m.set_option("conv_small14", v)
            feats = []
            for layer, shape in ((13, (B, 14, 14, 512)), (14, (B, 14, 14, 512)), (16, (B, 7, 7, 512))):
                f = torch.empty(*shape, dtype=torch.float16, device=DEV)
                _lib.check(lib.fac_debug_features_u8(m._ctx, x.data_ptr(), B, layer, f.data_ptr(), None), m._ctx, "dbg")
                feats.append(f.view(torch.int16).cpu())
            lg = m.forward_u8(x, pos_index=pidx)
            lg2 = m.forward_u8(x, pos_index=pidx)
            torch.cuda.synchronize()
            outs[v] = (feats, lg.cpu(), lg2.cpu())
    finally:
        m.set_option("conv_small14", 1)
    for a, b in zip(outs[0][0], outs[1][0]):
        assert torch.equal(a, b)
    assert torch.equal(outs[0][1], outs[1][1]) and torch.equal(outs[0][2], outs[1][2])


def test_direct_graph_follows_buffer_contents(models):
    """Small forwards on the same buffers as the previous call replay a graph
    captured on those buffers (no copies): each replay reads the crops the
    buffer holds at call time, and the logits / probabilities equal the eager
    forward's, through the first (copy-graph) call, the capture and later
    replays."""
    from fac_fake_amd import _lib
    lib = _lib.load()
    m = models["fp16"]
    B = 29
    x = torch.empty(B, 224, 224, 3, dtype=torch.uint8, device=DEV)
    pidx = (torch.arange(B) * 5 % 32).to(torch.int32).to(DEV)
    lg = torch.empty(B, 2, device=DEV)
    pr = torch.empty(B, 2, device=DEV)
    st = torch.cuda.current_stream().cuda_stream
    seeds = [11, 12, 11, 13, 12, 13]

    def run():
        out = []
        for s in seeds:
            x.copy_(torch.from_numpy(make_crops(B, seed=s)))
            _lib.check(lib.fac_forward_nhwc_u8(m._ctx, x.data_ptr(), B, pidx.data_ptr(), lg.data_ptr(), pr.data_ptr(),
                                               st), m._ctx, "forward")
            out.append((lg.clone(), pr.clone()))
        torch.cuda.synchronize()
        return out

    got = run()
    m.set_option("graph_max_b", 0)
    try:
        ref = run()
    finally:
        m.set_option("graph_max_b", 32)
    for s, (a, b) in zip(seeds, zip(got, ref)):
        assert torch.equal(a[0], b[0]) and torch.equal(a[1], b[1]), s
    assert not torch.equal(got[0][0], got[1][0])
