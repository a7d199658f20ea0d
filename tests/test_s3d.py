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
def test_emulation_within_16bit_envelope(golden, torch_threads, srm):
    from oracle import s3d_torch as O
    g = golden("s3d_golden.npz")
    x = torch.from_numpy(s3d_clips(2, 16, 112, seed=int(g["clip_seed"])))
    sd = make_s3d_state_dict(0, 1, srm == "yes")
    p_ref = torch.sigmoid(torch.from_numpy(g[f"logits_{srm}"]))
    for dt, tol in (("fp16", 1e-3), ("bf16", 1e-2)):
        p = torch.sigmoid(O.forward_emulated(sd, x, srm == "yes", dt))
        assert (p - p_ref).abs().max() <= tol, dt
