"""Generate the parity fixtures under tests/golden/ from the REFERENCE itself.

Runs only in the build container (it reads /root/reference, which does not
exist on the GPU box).  It imports ``CViT-main/model/cvit.py`` (plain torch +
einops, importable here), loads the repo's deterministic synthetic weights
(fac_fake_amd.weights, seed 0) and records the reference's outputs.  The
scoring helpers of ``cvit_prediction.py`` (which cannot be imported: it
chdirs to a Windows path and needs cv2/face_recognition at import) are
extracted with ``ast`` and executed on their own with torch only.

Fixtures (data only - inputs and outputs, no reference source):
  golden_c1.npz        1 crop (seed 1): logits, probs, per-layer stats
  golden_b32.npz       32 crops (seed 2), slots 0..31: logits
  golden_b256.npz      256 crops (seed 3) as 8 reference chunks of 32: logits
  golden_real.npz      2 real JPEG crops from CViT-main/sample_train_data: uint8 pixels + logits
  golden_chunks.npz    40 crops (seed 4) scored by predict()'s chunk rule: logits, video score
  golden_postproc.json pre_process_prediction(pred_sig(.)) on synthetic logits, N in {0..90}
  weights_checksums.json per-tensor (sum, abs-sum) of the synthetic state_dict (seed 0)
"""
from __future__ import annotations

import ast
import json
import os
import sys
from pathlib import Path

sys.dont_write_bytecode = True
REPO = Path(__file__).resolve().parents[1]
REF = Path("/root/reference/CViT-main")
OUT = REPO / "tests" / "golden"
sys.path.insert(0, str(REPO))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from fac_fake_amd.weights import make_crops, make_state_dict, state_dict_checksums  # noqa: E402

SAMPLE_IDX = np.array([0, 1, 7, 100, 1000, 4095, 5000, 12345, 25087, 33, 77, 2048, 999, 3, 64, 511])


def ref_model(sd):
    sys.path.insert(0, str(REF / "model"))
    from cvit import CViT  # the reference module
    m = CViT(image_size=224, patch_size=7, num_classes=2, channels=512, dim=1024, depth=6, heads=8, mlp_dim=2048)
    m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in sd.items()})
    return m.eval()


def ref_normalize(crops_u8):
    # cvit_prediction.py:209-215 (transforms.Normalize == (x - mean) / std on fp32 tensors)
    x = torch.tensor(crops_u8).float().permute((0, 3, 1, 2))
    mean = torch.tensor([0.485, 0.456, 0.406]).view(3, 1, 1)
    std = torch.tensor([0.229, 0.224, 0.225]).view(3, 1, 1)
    out = torch.empty_like(x)
    for i in range(len(x)):
        out[i] = (x[i] / 255. - mean) / std
    return out.contiguous()


def ref_scoring_helpers():
    src = (REF / "cvit_prediction.py").read_text(encoding="utf-8")
    tree = ast.parse(src)
    wanted = {"non_empty", "pred_sig", "pred_tensor", "pre_process_prediction"}
    fns = [n for n in tree.body if isinstance(n, ast.FunctionDef) and n.name in wanted]
    ns = {"torch": torch}
    exec(compile(ast.Module(body=fns, type_ignores=[]), "cvit_prediction_helpers", "exec"), ns)
    return ns


def stats(t: torch.Tensor):
    a = t.detach().permute(0, 2, 3, 1).reshape(-1).double() if t.dim() == 4 else t.detach().reshape(-1).double()
    idx = SAMPLE_IDX % a.numel()
    return np.array([a.sum().item(), (a * a).sum().item(), *a[idx].tolist()], np.float64)


@torch.no_grad()
def main():
    torch.set_num_threads(os.cpu_count() or 8)
    OUT.mkdir(parents=True, exist_ok=True)
    sd = make_state_dict(0)
    m = ref_model(sd)

    # C1: one crop, slot 0, with per-layer statistics of the NHWC activations
    crops = make_crops(1, seed=1)
    x = ref_normalize(crops)
    # block outputs (NHWC stats): after each ReLU, or after the MaxPool that follows it
    layer_out = []
    feats = list(m.features)
    h = x
    for i, mod in enumerate(feats):
        h = mod(h)
        nxt = feats[i + 1] if i + 1 < len(feats) else None
        if isinstance(mod, torch.nn.ReLU) and not isinstance(nxt, torch.nn.MaxPool2d):
            layer_out.append(stats(h))
        if isinstance(mod, torch.nn.MaxPool2d):
            layer_out.append(stats(h))
    logits = m(x)
    np.savez_compressed(OUT / "golden_c1.npz", crop_sum=np.int64(crops.astype(np.int64).sum()),
                        logits=logits.numpy(), probs=torch.sigmoid(logits).numpy(),
                        layer_stats=np.stack(layer_out), sample_idx=SAMPLE_IDX)

    # B=32, slots 0..31
    crops = make_crops(32, seed=2)
    logits = m(ref_normalize(crops))
    np.savez_compressed(OUT / "golden_b32.npz", crop_sum=np.int64(crops.astype(np.int64).sum()),
                        logits=logits.numpy())

    # B=256 as 8 chunks of 32 (config 2's crops; pos slot = j mod 32)
    crops = make_crops(256, seed=3)
    xs = ref_normalize(crops)
    logits = torch.cat([m(xs[i:i + 32]) for i in range(0, 256, 32)])
    np.savez_compressed(OUT / "golden_b256.npz", crop_sum=np.int64(crops.astype(np.int64).sum()),
                        logits=logits.numpy())

    # two real face crops from the reference's sample data (decoded with PIL)
    from PIL import Image
    paths = [REF / "sample_train_data/test/real/aaragvjucp_1.jpg",
             REF / "sample_train_data/test/fake/aavqiqgbzl_mjqktsbgyj_0.jpg"]
    real = np.stack([np.asarray(Image.open(p).convert("RGB").resize((224, 224)), dtype=np.uint8) for p in paths])
    logits = m(ref_normalize(real))
    np.savez_compressed(OUT / "golden_real.npz", crops=real, logits=logits.numpy(),
                        names=np.array([p.name for p in paths]))

    # predict()'s chunking on 40 crops: model(t[0:32]) then model(t[32:40]) (cvit_prediction.py:224-240)
    helpers = ref_scoring_helpers()
    crops = make_crops(40, seed=4)
    t = ref_normalize(crops)
    y = m(t[0:32])
    dft = helpers["non_empty"](t, 40, lower_bound=32, upper_bound=64, flag=True)
    y = helpers["pred_tensor"](y, m(dft))
    score = helpers["pre_process_prediction"](helpers["pred_sig"](y))
    np.savez_compressed(OUT / "golden_chunks.npz", crop_sum=np.int64(crops.astype(np.int64).sum()),
                        logits=y.numpy(), score=np.float32(score))

    # scoring table
    rng = np.random.default_rng(7)
    table = []
    for n in (1, 2, 3, 4, 5, 16, 29, 32, 33, 64, 90):
        lg = rng.normal(0, 2, size=(n, 2)).astype(np.float32)
        s = helpers["pre_process_prediction"](helpers["pred_sig"](torch.from_numpy(lg)))
        table.append({"n": n, "logits": lg.tolist(), "score": float(s)})
    # zero crops: predict() returns 0.5 before scoring (cvit_prediction.py:218-219)
    table.append({"n": 0, "logits": [], "score": 0.5})
    (OUT / "golden_postproc.json").write_text(json.dumps(table))

    (OUT / "weights_checksums.json").write_text(json.dumps(state_dict_checksums(sd)))
    print("wrote", sorted(p.name for p in OUT.iterdir()))


if __name__ == "__main__":
    main()
