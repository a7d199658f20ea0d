"""Generate the ResVitKan (BASELINE config 5) fixtures under tests/golden/ from
the REFERENCE itself.

Runs only in the build container (it reads /root/reference, which does not
exist on the GPU box).  It imports ``CViT-main/ResVitKan/ResVitKan.py`` (and
its ``kan.py``; plain torch + einops, importable here), loads the repo's
deterministic synthetic weights (fac_fake_amd.weights.make_resvitkan_state_dict,
seed 0) and records the reference's outputs.  Data only, no reference source:

  resvitkan_keys.json   the reference state_dict's keys and shapes, in order
  resvitkan_golden.npz  4 crops (make_crops seed 21, slots 0..3): stem-feature
                        and hidden-layer checksums, KAN layer-0 outputs, logits;
                        a KANLinear(2048, 64) on inputs spanning the whole
                        grid and beyond (seed 22): inputs and outputs
  resvitkan_golden_stages.npz
                        8 crops (make_crops seed 43, slots 0..7): logits and,
                        for the max-pool, each of the 16 Bottlenecks and bn2,
                        the per-channel mean over (H, W) of its output, plus
                        the 16-bit rounding envelope of each (the oracle's
                        emulation of the HIP path's rounding points vs the
                        reference), so a GPU test can localise a wrong block
"""
from __future__ import annotations

import json
import sys
from pathlib import Path

sys.dont_write_bytecode = True
REPO = Path(__file__).resolve().parents[1]
REF = Path("/root/reference/CViT-main/ResVitKan")
OUT = REPO / "tests" / "golden"
sys.path.insert(0, str(REPO))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from fac_fake_amd.weights import make_crops, make_resvitkan_state_dict, uniform  # noqa: E402
from tools.make_golden import ref_normalize  # noqa: E402


def main():
    torch.manual_seed(0)
    sys.path.insert(0, str(REF))
    import ResVitKan as R  # the reference module (imports kan.py from the same directory)
    sd = make_resvitkan_state_dict(0)
    m = R.CViT(image_size=224, patch_size=7, num_classes=2, channels=512, dim=1024, depth=6, heads=8,
               mlp_dim=2048).eval()
    ref_sd = m.state_dict()
    keys = [[k, list(v.shape)] for k, v in ref_sd.items()]
    (OUT / "resvitkan_keys.json").write_text(json.dumps(keys))
    m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in sd.items()})

    crops = make_crops(4, seed=21)
    x = ref_normalize(crops)
    feats, hid, kan0 = {}, {}, {}
    m.features.register_forward_hook(lambda mod, i, o: feats.__setitem__("f", o.detach().clone()))
    m.kan_head[2].register_forward_hook(lambda mod, i, o: hid.__setitem__("h", o.detach().clone()))
    hk = m.kan_head[3].layers[0].register_forward_hook(lambda mod, i, o: kan0.__setitem__("k", o.detach().clone()))
    with torch.no_grad():
        logits = m(x)
    hk.remove()
    f, h = feats["f"].numpy(), hid["h"].numpy()

    kl = m.kan_head[3].layers[0]
    kx = torch.from_numpy(uniform("kan_x", 8 * 2048, 22).reshape(8, 2048) * np.float32(2.6))
    with torch.no_grad():
        ky = kl(kx)
    np.savez_compressed(
        OUT / "resvitkan_golden.npz",
        crop_seed=np.int64(21), logits=logits.numpy(),
        feat_sum=np.float64(f.astype(np.float64).sum()), feat_abs=np.float64(np.abs(f).astype(np.float64).sum()),
        feat_sample=f.reshape(-1)[::9973].copy(),
        hidden_sum=np.float64(h.astype(np.float64).sum()), hidden_sample=h.reshape(-1)[::97].copy(),
        kan0=kan0["k"].numpy(), kan_x=kx.numpy(), kan_y=ky.numpy())
    print("logits", logits.numpy())
    print("feat range", f.min(), f.max(), "hidden range", h.min(), h.max())
    stages(m, sd)


def _rel(a, b):
    return float(np.abs(a - b).max() / (np.sqrt((b.astype(np.float64) ** 2).mean()) + 1e-30))


def stages(m, sd):
    from oracle import resvitkan_torch as O  # the rounding-point emulation, for the envelope only
    from oracle.cvit_torch import to_torch_sd
    seed, n = 43, 8
    x = ref_normalize(make_crops(n, seed=seed))
    taps = []
    f = m.features
    mods = [f.maxpool] + [blk for layer in (f.layer1, f.layer2, f.layer3, f.layer4) for blk in layer] + [f.bn2]
    hooks = [md.register_forward_hook(lambda mod, i, o: taps.append(o.detach().clone())) for md in mods]
    with torch.no_grad():
        logits = m(x).numpy()
    for hk in hooks:
        hk.remove()
    assert len(taps) == 18
    means = [t.double().mean(dim=(2, 3)).numpy() for t in taps]
    out = {"crop_seed": np.int64(seed), "n_crops": np.int64(n), "logits": logits}
    for i, mu in enumerate(means):
        out[f"mean_{i}"] = mu.astype(np.float32)
    tsd = to_torch_sd(sd)
    p_ref = 1 / (1 + np.exp(-logits.astype(np.float64)))
    for dt in ("fp16", "bf16"):
        et = []
        O.resnet50_emulated(tsd, x, dt, et)
        out[f"env_{dt}"] = np.array([_rel(t.double().mean(dim=(2, 3)).numpy(), mu) for t, mu in zip(et, means)])
        pe = torch.sigmoid(O.forward_emulated(tsd, x, dtype=dt)).double().numpy()
        out[f"env_prob_{dt}"] = np.float64(np.abs(pe - p_ref).max())
        print(dt, "env", np.round(out[f"env_{dt}"], 4), "prob", out[f"env_prob_{dt}"])
    print("probs", np.round(p_ref, 4))
    np.savez_compressed(OUT / "resvitkan_golden_stages.npz", **out)


if __name__ == "__main__":
    main()
