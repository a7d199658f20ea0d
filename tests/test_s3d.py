"""S3D (BASELINE config 4) on the CPU: the drop-in's state_dict layout and the
oracle pinned against outputs of the reference module itself
(tests/golden/s3d_*, tools/make_golden_s3d.py)."""
import numpy as np
import pytest
import torch

from fac_fake_amd.weights import make_s3d_state_dict, s3d_clips, s3d_param_specs


@pytest.mark.parametrize("srm", ["no", "yes"])
def test_param_specs_are_the_reference_layout(golden, srm):
    want = golden("s3d_keys.json")[srm]
    assert [[n, list(s)] for n, s, _ in s3d_param_specs(1, srm == "yes")] == want and len(want) == 465


def test_dropin_state_dict_layout(golden):
    from fac_fake_amd.s3d import S3D
    for srm in ("no", "yes"):
        m = S3D(1, srm)
        assert [[k, list(v.shape)] for k, v in m.state_dict().items()] == golden("s3d_keys.json")[srm]
        m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in make_s3d_state_dict(0, 1, srm == "yes").items()})


@pytest.mark.parametrize("srm", ["no", "yes"])
def test_oracle_matches_reference_goldens(golden, torch_threads, srm):
    from oracle import s3d_torch as O
    g = golden("s3d_golden.npz")
    x = torch.from_numpy(s3d_clips(2, 16, 112, seed=int(g["clip_seed"])))
    sd = make_s3d_state_dict(0, 1, srm == "yes")
    f = O.features_fp32(sd, x, srm == "yes").numpy()
    assert np.isclose(f.astype(np.float64).sum(), float(g[f"feat_sum_{srm}"]), rtol=1e-6)
    out = O.forward_fp32(sd, x, srm == "yes").numpy()
    assert np.abs(out - g[f"logits_{srm}"]).max() <= 1e-5


@pytest.mark.parametrize("srm", ["no", "yes"])
def test_oracle_matches_reference_at_harness_shape(golden, torch_threads, srm):
    """20 x 224 x 224 clips (S3D-test.py:130-190, model.py:344-354)."""
    from fac_fake_amd.weights import s3d_clips_varied
    from oracle import s3d_torch as O
    g = golden("s3d_golden_20x224.npz")
    x = torch.from_numpy(s3d_clips_varied(2, int(g["frames"]), int(g["size"]), seed=int(g["clip_seed"])))
    out = O.forward_fp32(make_s3d_state_dict(0, 1, srm == "yes"), x, srm == "yes").numpy()
    assert np.abs(out - g[f"logits_{srm}"]).max() <= 1e-5


@pytest.mark.parametrize("srm", ["no", "yes"])
def test_emulation_within_16bit_envelope(golden, torch_threads, srm):
    from oracle import s3d_torch as O
    g = golden("s3d_golden.npz")
    x = torch.from_numpy(s3d_clips(2, 16, 112, seed=int(g["clip_seed"])))
    sd = make_s3d_state_dict(0, 1, srm == "yes")
    p_ref = torch.sigmoid(torch.from_numpy(g[f"logits_{srm}"]))
    for dt, tol in (("fp16", 1e-3), ("bf16", 1e-2)):
        p = torch.sigmoid(O.forward_emulated(sd, x, srm == "yes", dt))
        assert (p - p_ref).abs().max() <= tol, dt


@pytest.mark.parametrize("srm", ["no", "yes"])
def test_oracle_every_block_matches_reference(golden, torch_threads, srm):
    """The oracle's base[i] outputs on the 8 content-varied clips: per-channel
    means equal to the reference module's (s3d_golden_blocks.npz) to fp32
    summation-order noise, and the fixture's logits spread (a fixture whose
    clips all score alike pins little)."""
    from oracle import s3d_torch as O
    from fac_fake_amd.weights import s3d_clips_varied
    g = golden("s3d_golden_blocks.npz")
    x = torch.from_numpy(s3d_clips_varied(int(g["n_clips"]), 16, 112, int(g["clip_seed"])))
    taps = []
    O.features_fp32(make_s3d_state_dict(0, 1, srm == "yes"), x, srm == "yes", taps)
    assert len(taps) == 16
    for i, t in enumerate(taps):
        got = t.double().mean(dim=(2, 3, 4)).numpy()
        ref = g[f"mean_{srm}_{i}"].astype(np.float64)
        assert np.abs(got - ref).max() <= 1e-5 * np.sqrt((ref ** 2).mean()) + 1e-7, i
    p = 1 / (1 + np.exp(-g[f"logits_{srm}"].astype(np.float64)))
    assert p.max() - p.min() > 0.03


def test_custom_round_semantics():
    """utils.py:25-38 (S3D harness): strict > 0.5 threshold; the first
    prediction above 0.5 wins, else the mean."""
    from fac_fake_amd.s3d import custom_round, custom_video_round
    assert list(custom_round([0.2, 0.5, 0.50001, 0.9])) == [0, 0, 1, 1]
    assert custom_video_round([0.1, 0.7, 0.9]) == 0.7
    assert abs(custom_video_round([0.1, 0.3]) - 0.2) < 1e-12
