"""ResVitKan (BASELINE config 5) on the CPU: the drop-in's state_dict layout and
the oracle pinned against outputs of the reference module itself
(tests/golden/resvitkan_*, tools/make_golden_resvitkan.py)."""
import numpy as np
import torch

from fac_fake_amd.weights import make_crops, make_resvitkan_state_dict, resvitkan_param_specs


def test_param_specs_are_the_reference_layout(golden):
    want = golden("resvitkan_keys.json")
    got = [[n, list(s)] for n, s, _ in resvitkan_param_specs()]
    assert got == want and len(got) == 408


def test_dropin_state_dict_layout(golden):
    from fac_fake_amd.resvitkan import ResVitKan
    m = ResVitKan()
    sd = m.state_dict()
    assert [[k, list(v.shape)] for k, v in sd.items()] == golden("resvitkan_keys.json")
    assert sd["features.bn1.num_batches_tracked"].dtype == torch.long
    # KAN grids are buffers holding the reference's initial knots (kan.py:39-48)
    g = golden("resvitkan_golden.npz")
    m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in make_resvitkan_state_dict(0).items()})
    from fac_fake_amd.weights import kan_grid
    grid = m.state_dict()["kan_head.3.layers.0.grid"]
    assert torch.equal(grid, torch.from_numpy(kan_grid(2048)))
    assert torch.allclose(grid[0], torch.linspace(-2.2, 2.2, 12), atol=1e-6)
    assert g["logits"].shape == (4, 2)


def test_oracle_matches_reference_goldens(golden, torch_threads):
    from oracle import resvitkan_torch as O
    from oracle.cvit_torch import normalize_u8, to_torch_sd
    g = golden("resvitkan_golden.npz")
    sd = to_torch_sd(make_resvitkan_state_dict(0))
    x = normalize_u8(make_crops(4, seed=int(g["crop_seed"])))
    f = O.resnet50_fp32(sd, x).numpy()
    assert np.isclose(f.astype(np.float64).sum(), float(g["feat_sum"]), rtol=1e-6)
    assert np.allclose(f.reshape(-1)[::9973], g["feat_sample"], rtol=1e-5, atol=1e-5)
    out = O.forward_fp32(sd, x).numpy()
    assert np.abs(out - g["logits"]).max() <= 1e-5
    ky = O.kan_linear_fp32(sd, "kan_head.3.layers.0", torch.from_numpy(g["kan_x"])).numpy()
    assert np.abs(ky - g["kan_y"]).max() <= 1e-6


def test_emulation_within_16bit_envelope(golden, torch_threads):
    """The HIP path's rounding points (emulated) stay near the fp32 reference:
    fp16 within the 1e-3 probability bar, bf16 within 1e-2."""
    from oracle import resvitkan_torch as O
    from oracle.cvit_torch import normalize_u8, to_torch_sd
    g = golden("resvitkan_golden.npz")
    sd = to_torch_sd(make_resvitkan_state_dict(0))
    x = normalize_u8(make_crops(4, seed=int(g["crop_seed"])))
    p_ref = torch.sigmoid(torch.from_numpy(g["logits"]))
    for dt, tol in (("fp16", 1e-3), ("bf16", 1e-2)):
        p = torch.sigmoid(O.forward_emulated(sd, x, dtype=dt))
        assert (p - p_ref).abs().max() <= tol, dt


def test_b_splines_partition_of_unity():
    """Inside the grid's interior the 8 cubic bases sum to 1 (kan.py:90-132)."""
    from oracle.resvitkan_torch import b_splines
    from fac_fake_amd.weights import kan_grid
    g = torch.from_numpy(kan_grid(4))
    x = torch.linspace(-0.99, 0.99, 40).view(10, 4)
    s = b_splines(x, g).sum(-1)
    assert torch.allclose(s, torch.ones_like(s), atol=1e-6)


def test_oracle_every_block_matches_reference(golden, torch_threads):
    """The oracle's max-pool, 16 Bottleneck and bn2 outputs on 8 crops: per-channel
    means equal to the reference module's (resvitkan_golden_stages.npz)."""
    from oracle import resvitkan_torch as O
    from oracle.cvit_torch import normalize_u8, to_torch_sd
    g = golden("resvitkan_golden_stages.npz")
    x = normalize_u8(make_crops(int(g["n_crops"]), seed=int(g["crop_seed"])))
    taps = []
    O.resnet50_fp32(to_torch_sd(make_resvitkan_state_dict(0)), x, taps)
    assert len(taps) == 18
    for i, t in enumerate(taps):
        got = t.double().mean(dim=(2, 3)).numpy()
        ref = g[f"mean_{i}"].astype(np.float64)
        assert np.abs(got - ref).max() <= 1e-5 * np.sqrt((ref ** 2).mean()) + 1e-7, i
