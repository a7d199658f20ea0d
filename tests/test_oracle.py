"""The oracle pinned against the reference's own outputs (tests/golden/, made by
tools/make_golden.py importing CViT-main/model/cvit.py).  CPU only."""
import numpy as np
import pytest
import torch

from fac_fake_amd.weights import make_crops, make_state_dict, state_dict_checksums
from oracle import cvit_numpy, postproc
from oracle.cvit_torch import forward_emulated, forward_fp32, normalize_u8


def _sig(x):
    return 1.0 / (1.0 + np.exp(-np.asarray(x, np.float64)))


def test_weight_generator_pinned(sd, golden):
    want = golden("weights_checksums.json")
    got = state_dict_checksums(sd)
    assert list(got) == list(want)          # 193 keys in the reference's order
    for k in want:
        assert got[k] == pytest.approx(want[k], rel=0, abs=0), k


def test_crop_generator_pinned(golden):
    for name, n, seed in (("golden_c1.npz", 1, 1), ("golden_b32.npz", 32, 2), ("golden_b256.npz", 256, 3),
                          ("golden_chunks.npz", 40, 4)):
        assert int(make_crops(n, seed).astype(np.int64).sum()) == int(golden(name)["crop_sum"]), name


def test_torch_oracle_c1(sd, golden, torch_threads):
    g = golden("golden_c1.npz")
    x = normalize_u8(make_crops(1, 1))
    out, feats = forward_fp32(sd, x, return_features=True)
    assert np.abs(out.numpy() - g["logits"]).max() <= 1e-5
    # per-block activation statistics (sum, sum of squares, 16 samples) of the reference
    for i, f in enumerate(feats):
        a = f.permute(0, 2, 3, 1).reshape(-1).double()
        s = g["layer_stats"][i]
        assert a.sum().item() == pytest.approx(s[0], rel=1e-5)
        assert (a * a).sum().item() == pytest.approx(s[1], rel=1e-5)
        idx = g["sample_idx"] % a.numel()
        np.testing.assert_allclose(a[idx].numpy(), s[2:], rtol=1e-4, atol=1e-5)


def test_torch_oracle_b32_and_real(sd, golden, torch_threads):
    g = golden("golden_b32.npz")
    out = forward_fp32(sd, normalize_u8(make_crops(32, 2)))
    assert np.abs(out.numpy() - g["logits"]).max() <= 1e-5
    r = golden("golden_real.npz")
    out = forward_fp32(sd, normalize_u8(r["crops"]))
    assert np.abs(out.numpy() - r["logits"]).max() <= 1e-5


def test_torch_oracle_b256_slots(sd, golden, torch_threads):
    """A 64-crop slice of config 2 with explicit slots j mod 32 (one call, two chunks' worth)."""
    g = golden("golden_b256.npz")
    crops = make_crops(256, 3)[64:128]
    out = forward_fp32(sd, normalize_u8(crops), pos_index=np.arange(64, 128) % 32)
    assert np.abs(out.numpy() - g["logits"][64:128]).max() <= 1e-5


def test_numpy_oracle_c1(sd, golden):
    """Independent numpy restatement (NHWC im2col) agrees with the reference."""
    g = golden("golden_c1.npz")
    x = cvit_numpy.normalize_u8(make_crops(1, 1))
    out = cvit_numpy.forward(sd, x)
    assert np.abs(out - g["logits"]).max() <= 2e-4
    assert np.abs(_sig(out) - g["probs"]).max() <= 1e-4


def test_chunk_rule_and_video_score(sd, golden, torch_threads):
    g = golden("golden_chunks.npz")
    crops = make_crops(40, 4)
    slots = postproc.chunk_slots(40)
    assert list(slots[:32]) == list(range(32)) and list(slots[32:]) == list(range(8))
    out = forward_fp32(sd, normalize_u8(crops), pos_index=slots).numpy()
    assert np.abs(out - g["logits"]).max() <= 1e-5
    assert postproc.video_score(out) == pytest.approx(float(g["score"]), abs=1e-6)


def test_postproc_table(golden):
    for row in golden("golden_postproc.json"):
        assert postproc.video_score(np.asarray(row["logits"], np.float32)) == pytest.approx(row["score"], abs=1e-6)


def test_product_scoring_helpers_match_reference_table(golden):
    from fac_fake_amd import prediction as P
    for row in golden("golden_postproc.json"):
        lg = torch.tensor(np.asarray(row["logits"], np.float32).reshape(-1, 2))
        s = P.pre_process_prediction(P.pred_sig(lg)) if row["n"] else torch.tensor(P.EMPTY_SCORE)
        assert float(s) == pytest.approx(row["score"], abs=1e-7), row["n"]
    for n in (0, 1, 31, 32, 33, 63, 64, 65, 89, 90, 120):
        assert list(P.chunk_slots(n)) == list(postproc.chunk_slots(n))
    t = torch.arange(100)
    assert P.non_empty(t, 100, 64, 90, True).tolist() == list(range(64, 90))
    assert P.non_empty(t, 70, 64, 90, True).tolist() == list(range(64, 70))
    assert P.non_empty(t, -1, -1, -1, False) is t


@pytest.mark.parametrize("dt,bound", [("fp16", 1e-3), ("bf16", 1e-2)])
def test_emulated_rounding_error_budget(sd, golden, dt, bound, torch_threads):
    """How far exact 16-bit operand rounding moves the fp32 reference."""
    g = golden("golden_b32.npz")
    em = forward_emulated(sd, normalize_u8(make_crops(32, 2)), dtype=dt).numpy()
    dp = np.abs(_sig(em) - _sig(g["logits"])).max()
    assert dp <= bound, dp


def test_seeded_generators_are_deterministic():
    a = make_state_dict(5)
    b = make_state_dict(5)
    assert all(np.array_equal(a[k], b[k]) for k in a)
    assert not np.array_equal(make_crops(1, 1), make_crops(1, 2))
