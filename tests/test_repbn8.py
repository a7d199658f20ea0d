"""CViT RepBn8 variant.

CPU: the drop-in's state_dict layout and its host-side DEConv fold against
the reference's own class code (tests/golden/repbn8_*,
tools/make_golden_repbn8.py), the oracle pinned bit-exactly to the same
goldens, and the 16-bit rounding envelope of the HIP path's arithmetic.

GPU (marked): GGCA kernel vs the oracle's GGCA on the same 16-bit features;
the conv stack vs the oracle's emulation; end-to-end logits vs the
reference's fp32 goldens within the emulation's own envelope (the variant
squares its features in x * GGCA(x), so 16-bit rounding moves its
probabilities further than the plain CViT's: emulated fp16 1.9e-3, bf16
1.1e-2 on these weights); uint8 == fp32-NCHW input paths; graph replay.
"""
import numpy as np
import pytest
import torch

from fac_fake_amd.weights import make_crops, make_repbn8_state_dict, repbn8_param_specs

DEV = "cuda:0"
# probability tolerances vs the fp32 reference: 2x the emulated rounding envelope
TOL = {"fp16": 4e-3, "bf16": 2.5e-2}


def _sd_t():
    return {k: torch.from_numpy(np.asarray(v)) for k, v in make_repbn8_state_dict(0).items()}


def test_param_specs_are_the_reference_layout(golden):
    want = golden("repbn8_keys.json")
    got = [[n, list(s)] for n, s, _ in repbn8_param_specs()]
    assert got == want and len(got) == 359


def test_dropin_state_dict_layout(golden):
    from fac_fake_amd.repbn8 import CViT
    m = CViT()
    sd = m.state_dict()
    assert [[k, list(v.shape)] for k, v in sd.items()] == golden("repbn8_keys.json")
    assert int(sd["transformer.layers.0.1.fn.norm.total_step"]) == 300000
    m.load_state_dict(_sd_t())
    with pytest.raises(RuntimeError):
        m.train()
    with pytest.raises(RuntimeError):          # no CPU fallback
        m(torch.zeros(1, 3, 224, 224))


def test_host_deconv_fold_is_the_reference_algebra(golden):
    """The drop-in folds DEConv on the host with the reference's tensor ops:
    bit-identical to DEConv.forward's w, b (:329-338) as the reference computes them."""
    from fac_fake_amd.repbn8 import deconv_fold
    g = golden("repbn8_golden.npz")
    w, b = deconv_fold(_sd_t(), "features1.3")
    assert np.array_equal(w.numpy(), g["deconv_w"]) and np.array_equal(b.numpy(), g["deconv_b"])


def test_oracle_matches_reference_goldens(golden, torch_threads):
    from oracle import repbn8_torch as O
    from oracle.cvit_torch import normalize_u8
    g = golden("repbn8_golden.npz")
    x = normalize_u8(make_crops(4, seed=int(g["crop_seed"])))
    out, f2, wt = O.forward_fp32(make_repbn8_state_dict(0), x, return_features=True)
    assert np.abs(out.numpy() - g["logits"]).max() <= 1e-5   # CPU BLAS differs across hosts
    assert np.isclose(f2.double().sum().item(), float(g["f2_sum"]), rtol=1e-6)
    assert np.isclose(wt.double().sum().item(), float(g["weighted_sum"]), rtol=1e-6)
    assert np.allclose(wt.numpy().reshape(-1)[::997], g["weighted_sample"], rtol=1e-5, atol=1e-6)


def test_emulation_envelope(golden, torch_threads):
    """The HIP path's rounding points (emulated) against the fp32 reference:
    half the GPU tolerance, so the tolerance leaves room for accumulation order."""
    from oracle import repbn8_torch as O
    from oracle.cvit_torch import normalize_u8
    g = golden("repbn8_golden.npz")
    x = normalize_u8(make_crops(4, seed=int(g["crop_seed"])))
    p_ref = torch.sigmoid(torch.from_numpy(g["logits"]))
    for dt in ("fp16", "bf16"):
        p = torch.sigmoid(O.forward_emulated(make_repbn8_state_dict(0), x, dtype=dt))
        assert (p - p_ref).abs().max() <= TOL[dt] / 2, dt


# ---------------------------------------------------------------- GPU
@pytest.fixture(scope="module")
def rb8():
    assert torch.cuda.is_available(), "GPU tests need a visible MI355X"
    from fac_fake_amd.repbn8 import CViT
    out = {}
    for dt in ("fp16", "bf16"):
        m = CViT(dtype=dt)
        m.load_state_dict(_sd_t())
        m.to(DEV)
        out[dt] = m
    return out


@pytest.mark.gpu
@pytest.mark.parametrize("dt", ["fp16", "bf16"])
def test_repbn8_matches_reference(rb8, golden, dt):
    g = golden("repbn8_golden.npz")
    crops = torch.from_numpy(make_crops(4, seed=int(g["crop_seed"]))).to(DEV)
    with torch.no_grad():
        lg, pr = rb8[dt].forward_u8(crops, return_probs=True)
    torch.cuda.synchronize()
    p_ref = 1 / (1 + np.exp(-g["logits"]))
    assert np.abs(pr.cpu().numpy() - p_ref).max() <= TOL[dt]
    assert np.allclose(pr.cpu().numpy(), 1 / (1 + np.exp(-lg.cpu().numpy())), atol=1e-6)


@pytest.mark.gpu
def test_repbn8_u8_and_nchw_paths_agree(rb8):
    from oracle.cvit_torch import normalize_u8
    crops = make_crops(3, seed=33)
    m = rb8["fp16"]
    with torch.no_grad():
        a = m.forward_u8(torch.from_numpy(crops).to(DEV))
        b = m(normalize_u8(crops).to(DEV))
    torch.cuda.synchronize()
    assert torch.equal(a, b)


@pytest.mark.gpu
def test_ggca_kernel_vs_oracle(rb8, torch_threads):
    """fac_ggca on 16-bit features against the oracle's GGCA (fp32, reference
    op order) on the same values: x * ((x * att_h) * att_w) within one 16-bit
    rounding of the output."""
    from oracle import repbn8_torch as O
    from oracle.cvit_torch import to_torch_sd
    m = rb8["fp16"]
    gen = torch.Generator().manual_seed(5)
    f = (torch.rand(6, 1, 7, 7, 512, generator=gen) * 3).to(torch.float16)
    got = m.weighted_features16(f.to(DEV)).float().cpu()
    xf = f.float()[:, 0].permute(0, 3, 1, 2)
    ref = (xf * O.ggca(to_torch_sd(make_repbn8_state_dict(0)), xf)).permute(0, 2, 3, 1).unsqueeze(1)
    err = (got - ref).abs() / ref.abs().clamp_min(1e-3)
    assert float(err.max()) <= 2 ** -10 + 1e-5


@pytest.mark.gpu
def test_repbn8_features_match_emulation(rb8, torch_threads):
    """The 18-conv stack (DEConv and BN folded, ReLU only where the reference
    has one) against the oracle's emulation of the same rounding points."""
    from oracle import repbn8_torch as O
    from oracle.cvit_torch import normalize_u8
    crops = make_crops(2, seed=34)
    m = rb8["fp16"]
    with torch.no_grad():
        m.forward_u8(torch.from_numpy(crops).to(DEV))   # prepares the packed layers
        f = m.features(torch.from_numpy(crops).to(DEV), u8=True).float().cpu()
    _, ref, _ = O.forward_emulated(make_repbn8_state_dict(0), normalize_u8(crops), dtype="fp16", return_features=True)
    ref = ref.permute(0, 2, 3, 1)
    rel = float((f - ref).norm() / ref.norm())
    assert rel <= 5e-3, rel


@pytest.mark.gpu
def test_repbn8_graph_replay_matches_eager(rb8):
    m = rb8["bf16"]
    crops = torch.from_numpy(make_crops(8, seed=35)).to(DEV)
    slots = torch.arange(8, dtype=torch.int32, device=DEV) * 3 % 32
    with torch.no_grad():
        eager = m.forward_u8(crops, pos_index=slots)
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        g = torch.cuda.CUDAGraph()
        with torch.cuda.stream(s):
            m.forward_u8(crops, pos_index=slots)
            with torch.cuda.graph(g, stream=s):
                out = m.forward_u8(crops, pos_index=slots)
        g.replay()
    torch.cuda.synchronize()
    assert torch.equal(out, eager)
