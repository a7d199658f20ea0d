"""Host-side checks that need no GPU: the C ABI library and the Python mirror."""
import ctypes
import re
from pathlib import Path

import numpy as np
import pytest
import torch

REPO = Path(__file__).resolve().parents[1]


def _header_symbols():
    text = "".join(h.read_text() for h in sorted((REPO / "include").glob("*.h")))
    return sorted(set(re.findall(r"\b(fac_[a-z0-9_]+)\s*\(", text)))


def test_header_declares_the_abi():
    syms = _header_symbols()
    for s in ("fac_create", "fac_load_weights", "fac_forward_nchw_f32", "fac_forward_nhwc_u8", "fac_destroy",
              "fac_last_error", "fac_reserve", "fac_video_score"):
        assert s in syms


def test_library_loads_and_exports_every_symbol(built_lib):
    lib = ctypes.CDLL(str(built_lib))
    for s in _header_symbols():
        assert hasattr(lib, s), s
    from fac_fake_amd import _lib
    assert set(_header_symbols()) == set(_lib.SIGNATURES)


def test_library_is_gfx950_code(built_lib):
    data = built_lib.read_bytes()
    assert b"gfx950" in data
    assert b"__hip_fatbin" in data or b"HIPF" in data or b"__CLANG_OFFLOAD_BUNDLE__" in data


def test_version_and_null_safety(built_lib):
    from fac_fake_amd import _lib
    lib = _lib.load()
    assert lib.fac_version().decode().startswith("fac_cvit")
    assert lib.fac_create(0, 7, None) == -1                       # bad dtype / null out
    assert lib.fac_load_weights(None, None, 0) == -1
    assert lib.fac_forward_nhwc_u8(None, None, 1, None, None, None, None) == -1
    assert lib.fac_last_error(None) == b"null context"
    lib.fac_destroy(None)


def test_conv_nd_dual_argument_checks(built_lib):
    """fac_conv_nd_dual rejects bad descriptors before touching the GPU: null
    pointers / mixed dtypes / a residual flag (FAC_ERR_ARG), a non-uniform-tap
    cin or mismatched output positions (FAC_ERR_SHAPE)."""
    import ctypes as C
    from fac_fake_amd import _lib
    from fac_fake_amd.ops import ConvDesc
    lib = _lib.load()
    assert lib.fac_conv_nd_dual(None, None, None) == -1

    def desc(cin, h, s, cout=256):
        d = ConvDesc()
        d.dtype, d.inp, d.weight, d.out = 0, 16, 16, 16
        d.n, d.d, d.h, d.w, d.cin, d.cout = 2, 1, h, h, cin, cout
        d.kd = d.kh = d.kw = 1
        d.sd, d.sh, d.sw = 1, s, s
        d.od, d.oh, d.ow = 1, (h - 1) // s + 1, (h - 1) // s + 1
        d.k_pad = (cin + 63) // 64 * 64
        d.ldo = cout
        return d

    a, b = desc(128, 28, 1), desc(256, 56, 2)
    bad = desc(128, 28, 1)
    bad.dtype = 1
    assert lib.fac_conv_nd_dual(C.byref(bad), C.byref(b), None) == -1          # mixed dtypes
    r = desc(128, 28, 1)
    r.flags = 2                                                                   # FAC_CONV_RESID
    assert lib.fac_conv_nd_dual(C.byref(r), C.byref(b), None) == -1
    for f in (8, 16, 32, 1 | 16):                      # OUT_F32, MAXPOOL3S2, an undefined bit, RELU | MAXPOOL3S2
        r.flags = f
        assert lib.fac_conv_nd_dual(C.byref(r), C.byref(b), None) == -1, f
    assert lib.fac_conv_nd_dual(C.byref(desc(96, 28, 1)), C.byref(b), None) == -2  # cin % 64
    assert lib.fac_conv_nd_dual(C.byref(a), C.byref(desc(256, 56, 1)), None) == -2  # 56x56 vs 28x28 outputs
    assert lib.fac_conv_nd_dual(C.byref(a), C.byref(desc(256, 56, 2, cout=128)), None) == -2  # cout differs


def test_conv_maxpool_flag_argument_checks(built_lib):
    """FAC_CONV_MAXPOOL3S2 is only accepted on the space-to-depth first conv
    with FAC_CONV_RELU alone; anything else is FAC_ERR_ARG, returned before
    any launch."""
    import ctypes as C
    from fac_fake_amd import _lib
    from fac_fake_amd.ops import ConvDesc, MAXPOOL3S2, RELU, RESID
    lib = _lib.load()

    def desc(kh=4, cin=16, cout=64, h=115, flags=RELU | MAXPOOL3S2):
        d = ConvDesc()
        d.dtype, d.inp, d.weight, d.out = 0, 16, 16, 16
        d.n, d.d, d.h, d.w, d.cin, d.cout = 2, 1, h, h, cin, cout
        d.kd, d.kh, d.kw = 1, kh, kh
        d.sd = d.sh = d.sw = 1
        d.od, d.oh, d.ow = 1, h - kh + 1, h - kh + 1
        d.k_pad = (kh * kh * cin + 63) // 64 * 64
        d.ldo, d.flags = cout, flags
        return d

    assert lib.fac_conv_nd(C.byref(desc(flags=MAXPOOL3S2)), None) == -1            # no ReLU
    assert lib.fac_conv_nd(C.byref(desc(flags=RELU | RESID | MAXPOOL3S2)), None) == -1
    assert lib.fac_conv_nd(C.byref(desc(kh=3, cin=64)), None) == -1                # not the s2d conv
    assert lib.fac_conv_nd(C.byref(desc(cout=128)), None) == -1
    assert lib.fac_conv_nd(C.byref(desc(h=60)), None) == -1                        # 57 outputs: no 8 x 28 boxes


def test_bottleneck_pw2_argument_checks(built_lib):
    """fac_bottleneck_pw2 rejects null / mismatched descriptors before any
    launch: FAC_ERR_ARG for pointers, dtypes and flags, FAC_ERR_SHAPE for
    widths and positions."""
    import ctypes as C
    from fac_fake_amd import _lib
    from fac_fake_amd.ops import ConvDesc, RELU, RELU2, RESID
    lib = _lib.load()
    assert lib.fac_bottleneck_pw2(None, None, None) == -1

    def desc(cin, cout, flags, h=56):
        d = ConvDesc()
        d.dtype, d.inp, d.weight, d.bias, d.out, d.residual = 0, 16, 16, 16, 16, 16
        d.n, d.d, d.h, d.w, d.cin, d.cout = 2, 1, h, h, cin, cout
        d.kd = d.kh = d.kw = d.sd = d.sh = d.sw = 1
        d.od, d.oh, d.ow = 1, h, h
        d.k_pad = (cin + 63) // 64 * 64
        d.ldo, d.ldr, d.flags = cout, 256, flags
        return d

    c3, c1 = desc(64, 256, RELU | RESID | RELU2), desc(256, 64, RELU)
    assert lib.fac_bottleneck_pw2(C.byref(desc(64, 256, RELU | RESID)), C.byref(c1), None) == -1   # no RELU2
    assert lib.fac_bottleneck_pw2(C.byref(c3), C.byref(desc(256, 64, 0)), None) == -1              # conv1 without ReLU
    assert lib.fac_bottleneck_pw2(C.byref(desc(128, 256, RELU | RESID | RELU2)), C.byref(c1), None) == -2
    assert lib.fac_bottleneck_pw2(C.byref(c3), C.byref(desc(256, 256, RELU)), None) == -2          # conv1 width
    assert lib.fac_bottleneck_pw2(C.byref(c3), C.byref(desc(256, 64, RELU, h=28)), None) == -2     # positions differ


def test_state_dict_is_the_reference_layout(golden):
    from fac_fake_amd.cvit import CViT
    want = list(golden("weights_checksums.json"))
    m = CViT()
    sd = m.state_dict()
    assert list(sd) == want
    assert sd["features.1.num_batches_tracked"].dtype == torch.long
    assert tuple(sd["patch_to_embedding.weight"].shape) == (1024, 25088)
    assert tuple(sd["pos_embedding"].shape) == (32, 1, 1024)


def test_load_state_dict_roundtrip(sd):
    from fac_fake_amd.cvit import CViT
    m = CViT(dtype="fp16")
    m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in sd.items()})
    got = m.state_dict()
    assert all(np.array_equal(got[k].numpy(), np.asarray(sd[k])) for k in sd)
    with pytest.raises(RuntimeError):
        m.load_state_dict({"pos_embedding": torch.zeros(32, 1, 1024)})   # strict, like nn.Module


def test_weight_versions_follow_replaced_submodules():
    """the drop-ins' weight-change check caches its parameter
    slots; replacing a submodule after the first call (or updating a weight in
    place, or swapping a tensor) must still change the versions tuple."""
    from fac_fake_amd.cvit import CViT, weight_versions
    m = CViT()
    v0 = weight_versions(m)
    assert weight_versions(m) == v0
    head0 = getattr(m.mlp_head, "0")
    with torch.no_grad():
        head0.weight.add_(1.0)                                                  # in place
    v1 = weight_versions(m)
    assert v1 != v0
    head0.weight = torch.nn.Parameter(head0.weight.detach().clone())            # swapped tensor
    v2 = weight_versions(m)
    assert v2 != v1
    out_f, in_f = head0.weight.shape
    setattr(m.mlp_head, "0", torch.nn.Linear(in_f, out_f))                      # replaced submodule
    v3 = weight_versions(m)
    assert v3 != v2 and len(v3) == len(v2)
    assert weight_versions(m) == v3


def test_constructor_contract():
    from fac_fake_amd.cvit import CViT
    with pytest.raises(AssertionError):
        CViT(image_size=225)
    with pytest.raises(NotImplementedError):
        CViT(depth=4)
    with pytest.raises(ValueError):
        CViT(dtype="fp8")
    m = CViT()
    assert not m.training
    with pytest.raises(RuntimeError):
        m.train()


def test_forward_fails_loudly_without_gpu():
    from fac_fake_amd.cvit import CViT
    m = CViT()
    with pytest.raises(RuntimeError):
        m(torch.zeros(1, 3, 224, 224))
    with pytest.raises(RuntimeError):   # a mask does not change that (no CPU fallback)
        m(torch.zeros(1, 3, 224, 224), mask=torch.ones(1, 1, dtype=torch.bool))
    with pytest.raises(ValueError):
        m(torch.zeros(1, 3, 112, 112))


def test_pos_index_rules():
    from fac_fake_amd.cvit import CViT
    p = CViT._pos_index(5, None, "cpu")
    assert p.tolist() == [0, 1, 2, 3, 4] and p.dtype == torch.int32
    with pytest.raises(RuntimeError, match="must match"):
        CViT._pos_index(33, None, "cpu")
    with pytest.raises(IndexError):
        CViT._pos_index(2, [0, 32], "cpu")
    with pytest.raises(ValueError):
        CViT._pos_index(2, [0], "cpu")
    assert CViT._pos_index(40, np.arange(40) % 32, "cpu").tolist()[32:] == list(range(8))


def test_drop_in_import_path():
    """`sys.path.insert(1, 'model'); from cvit import CViT` resolves to the HIP module."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("cvit_dropin", REPO / "model" / "cvit.py")
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    from fac_fake_amd.cvit import CViT
    assert mod.CViT is CViT


def test_sharding_bounds():
    from fac_fake_amd.sharding import shard_bounds
    for n in (0, 1, 7, 29, 300, 301):
        for w in (1, 2, 3, 8):
            spans = [shard_bounds(n, w, r) for r in range(w)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
            sizes = [hi - lo for lo, hi in spans]
            assert max(sizes) - min(sizes) <= 1


@pytest.mark.parametrize("H,ci,co", [(224, 32, 32), (112, 64, 64), (56, 128, 128), (28, 256, 256), (14, 512, 512)])
def test_conv3x3_weight_packing_layout(built_lib, H, ci, co):
    """fac_conv3x3_pack (host code, stack_ops.hip): [n-block][chunk][tap][q][BN][8]
    with BN = conv_block_n(H); below 224 the 16-byte pieces of the odd-kernel-row
    taps are stored as q ^ 2, matching conv.hip's row-parity-swizzled halo."""
    from fac_fake_amd import _lib
    lib = _lib.load()
    bn = {224: 32, 112: 64, 56: 128, 28: 256, 14: 128}[H]
    n = lib.fac_conv3x3_packed_elems(H, ci, co)
    assert n == co * ci * 9
    w = (torch.arange(co * ci * 9, dtype=torch.float32) % 2039).reshape(co, ci, 3, 3) / 1024.0
    out = torch.empty(n, dtype=torch.int16)
    _lib.check(lib.fac_conv3x3_pack(1, H, ci, co, w.data_ptr(), out.data_ptr()), None, "pack")  # fp16: exact here
    got = out.view(torch.float16).float().reshape(co // bn, ci // 32, 9, 4, bn, 8)
    for nb in range(co // bn):
        for ch in range(ci // 32):
            for t in range(9):
                for q in range(4):
                    qs = q ^ 2 if (H != 224 and (t // 3) % 2 == 1) else q
                    want = w[nb * bn:(nb + 1) * bn, ch * 32 + qs * 8:ch * 32 + qs * 8 + 8].reshape(bn, 8, 9)[:, :, t]
                    assert torch.equal(got[nb, ch, t, q], want), (nb, ch, t, q)


def test_reference_mask_semantics(golden):
    """cvit.py:50-55's mask=: the host check reproduces the reference's
    errors (AssertionError for a wrong width, the broadcast RuntimeError for
    B not in {1, heads}) and which masks poison the logits with NaN
    (tests/golden/mask_semantics.json, tools/make_golden_mask.py)."""
    import torch
    from fac_fake_amd.cvit import reference_mask_poisons
    for c in golden("mask_semantics.json"):
        mask = torch.tensor(c["mask"], dtype=torch.bool)
        if c["outcome"] == "error":
            exc = {"AssertionError": AssertionError, "RuntimeError": RuntimeError}[c["error"]]
            with pytest.raises(exc):
                reference_mask_poisons(mask, c["B"])
        else:
            assert reference_mask_poisons(mask, c["B"]) == (c["outcome"] == "nan"), c
            if c["outcome"] == "nan":
                assert all(c["nan_rows"])


def test_segmented_score_argument_checks(built_lib):
    """fac_video_score_seg rejects a negative count and null buffers, and an
    empty segment list is a no-op; none of these cases touches the device."""
    from fac_fake_amd import _lib
    lib = _lib.load()
    assert lib.fac_video_score_seg(None, None, -1, None, None) == -1
    assert lib.fac_video_score_seg(None, None, 0, None, None) == 0
    assert lib.fac_video_score_seg(None, None, 2, None, None) == -1
