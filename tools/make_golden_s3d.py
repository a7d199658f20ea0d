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

from fac_fake_amd.weights import make_s3d_state_dict, s3d_clips  # noqa: E402


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


if __name__ == "__main__":
    main()
