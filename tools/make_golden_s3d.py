"""Generate the S3D (BASELINE config 4) fixtures under tests/golden/ from the
REFERENCE itself.

Runs only in the build container (it reads /root/reference, which does not
exist on the GPU box).  It imports ``sx_exp_deepfakedetect-master/S3D/model.py``
(with its ``SRM`` package; plain torch + numpy, importable here), loads the
repo's deterministic synthetic weights (fac_fake_amd.weights.make_s3d_state_dict,
seed 0, num_class 1) and records the reference's outputs.  Data only:

  s3d_keys.json       the reference state_dict's keys and shapes (SRM_net 'no'
                      and 'yes'), in order
  s3d_golden.npz      2 clips of 16 x 112 x 112 raw 0..255 pixels (s3d_clips,
                      seed 31) through S3D(1, 'no') and S3D(1, 'yes'): logits
                      and a checksum of the base features
  s3d_golden_blocks.npz
                      8 content-varied clips (s3d_clips_varied, seed 41)
                      through S3D(1, 'no') and S3D(1, 'yes'): logits and, for
                      every base[i] (the Mixed_* blocks included), the
                      per-channel mean over (T, H, W) of its output; plus the
                      16-bit rounding envelope of each (the oracle's emulation
                      of the HIP path's rounding points vs the reference), so
                      the GPU tests can localise a wrong branch or channel
                      slot that a single logit per clip would hide
"""
from __future__ import annotations

import json
import sys
from pathlib import Path

sys.dont_write_bytecode = True
REPO = Path(__file__).resolve().parents[1]
REF = Path("/root/reference/sx_exp_deepfakedetect-master/S3D")
OUT = REPO / "tests" / "golden"
sys.path.insert(0, str(REPO))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from fac_fake_amd.weights import make_s3d_state_dict, s3d_clips, s3d_clips_varied  # noqa: E402


def main():
    sys.path.insert(0, str(REF))
    from model import S3D  # the reference module (imports SRM/HPF.py from the same directory)
    keys, out = {}, {}
    x = torch.from_numpy(s3d_clips(2, 16, 112, seed=31))
    for srm in ("no", "yes"):
        m = S3D(1, srm).eval()
        keys[srm] = [[k, list(v.shape)] for k, v in m.state_dict().items()]
        sd = make_s3d_state_dict(0, 1, srm == "yes")
        m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in sd.items()})
        feats = {}
        m.base.register_forward_hook(lambda mod, i, o: feats.__setitem__("f", o.detach().clone()))
        with torch.no_grad():
            lg = m(x)
        f = feats["f"].numpy()
        out[f"logits_{srm}"] = lg.numpy()
        out[f"feat_sum_{srm}"] = np.float64(f.astype(np.float64).sum())
        out[f"feat_abs_{srm}"] = np.float64(np.abs(f).astype(np.float64).sum())
        print(srm, lg.numpy().ravel(), "feat range", f.min(), f.max())
    (OUT / "s3d_keys.json").write_text(json.dumps(keys))
    np.savez_compressed(OUT / "s3d_golden.npz", clip_seed=np.int64(31), **out)
    blocks(S3D)


def _rel(a, b):
    """max |a - b| over everything, relative to the rms of b."""
    return float(np.abs(a - b).max() / (np.sqrt((b.astype(np.float64) ** 2).mean()) + 1e-30))


def blocks(S3D):
    from oracle import s3d_torch as O  # the rounding-point emulation, for the envelope only
    seed, n = 41, 8
    x = torch.from_numpy(s3d_clips_varied(n, 16, 112, seed))
    out = {"clip_seed": np.int64(seed), "n_clips": np.int64(n)}
    for srm in ("no", "yes"):
        m = S3D(1, srm).eval()
        sd = make_s3d_state_dict(0, 1, srm == "yes")
        m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in sd.items()})
        taps = []
        hooks = [m.base[i].register_forward_hook(lambda mod, i_, o: taps.append(o.detach().clone()))
                 for i in range(len(m.base))]
        with torch.no_grad():
            lg = m(x).numpy()
        for h in hooks:
            h.remove()
        means = [t.double().mean(dim=(2, 3, 4)).numpy() for t in taps]
        out[f"logits_{srm}"] = lg
        for i, mu in enumerate(means):
            out[f"mean_{srm}_{i}"] = mu.astype(np.float32)
        p_ref = 1 / (1 + np.exp(-lg.astype(np.float64)))
        for dt in ("fp16", "bf16"):
            et = []
            O.features_emulated(sd, x, srm == "yes", dt, et)
            out[f"env_{srm}_{dt}"] = np.array([_rel(t.double().mean(dim=(2, 3, 4)).numpy(), mu)
                                              for t, mu in zip(et, means)])
            pe = torch.sigmoid(O.forward_emulated(sd, x, srm == "yes", dt)).double().numpy()
            out[f"env_prob_{srm}_{dt}"] = np.float64(np.abs(pe - p_ref).max())
        print(srm, "probs", np.round(p_ref.ravel(), 4), "env fp16", np.round(out[f"env_{srm}_fp16"], 4),
              "bf16", np.round(out[f"env_{srm}_bf16"], 4), out[f"env_prob_{srm}_fp16"], out[f"env_prob_{srm}_bf16"])
    np.savez_compressed(OUT / "s3d_golden_blocks.npz", **out)


def harness_shape(S3D):
    """The reference harness's clip shape (S3D-test.py:130-190 reads 200
    frames and keeps every 10th: 20 frames; model.py:344-354 profiles
    20 x 224 x 224): 2 raw clips of 20 x 224 x 224 (s3d_clips_varied, seed 37)
    through S3D(1, 'no') and S3D(1, 'yes') -> s3d_golden_20x224.npz (logits,
    plus each variant's emulated 16-bit rounding envelope in probability)."""
    from oracle import s3d_torch as O
    x = torch.from_numpy(s3d_clips_varied(2, 20, 224, seed=37))
    out = {"clip_seed": np.int64(37), "frames": np.int64(20), "size": np.int64(224)}
    for srm in ("no", "yes"):
        m = S3D(1, srm).eval()
        sd = make_s3d_state_dict(0, 1, srm == "yes")
        m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in sd.items()})
        with torch.no_grad():
            lg = m(x).numpy()
        out[f"logits_{srm}"] = lg
        p_ref = 1 / (1 + np.exp(-lg.astype(np.float64)))
        for dt in ("fp16", "bf16"):
            pe = torch.sigmoid(O.forward_emulated(sd, x, srm == "yes", dt)).double().numpy()
            out[f"env_prob_{srm}_{dt}"] = np.float64(np.abs(pe - p_ref).max())
        print(srm, "20x224 probs", np.round(p_ref.ravel(), 5), out[f"env_prob_{srm}_fp16"], out[f"env_prob_{srm}_bf16"])
    np.savez_compressed(OUT / "s3d_golden_20x224.npz", **out)


if __name__ == "__main__":
    if "--harness-shape" in sys.argv:
        sys.path.insert(0, str(REF))
        from model import S3D as _S3D  # the reference module
        harness_shape(_S3D)
    else:
        main()
