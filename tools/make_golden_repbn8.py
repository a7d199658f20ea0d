"""Generate the CViT RepBn8 fixtures under tests/golden/ from
the REFERENCE's own class code.

Runs only in the build container (it reads /root/reference, which does not
exist on the GPU box).  ``CViT-main/model/cvit_GGCA_ADD_DEConv_RepBn8.py``
cannot be imported as a module here: line 7 imports ``torchsummary`` (not in
the image; only its ``__main__`` block uses it) and the module is CUDA-only —
``Conv2d_vd.__init__`` calls ``self.conv.cuda()`` (:302) and every
``get_weight`` allocates its zero-filled scratch with
``torch.cuda.FloatTensor(...).fill_(0)`` (:226, :294, :312).  So this script
parses the file with ``ast``, keeps its import statements except
``torchsummary``, its module-level assignments (``ln``, ``linearnorm``) and
every class definition, unchanged, and executes them with two substitutions
that do not touch the arithmetic:

  * ``torch.cuda.FloatTensor(*shape)`` -> a CPU fp32 tensor of that shape
    (the code ``fill_(0)``s it and overwrites slices; only the device differs)
  * ``nn.Conv1d.cuda()`` -> returns the module unchanged (stays on the CPU)

Everything else — DEConv's weight algebra, GGCA, LinearNorm's eval branch,
the transformer, the head — is the reference's code on PyTorch CPU.  The
fixtures are data only (no reference source):

  repbn8_keys.json   the reference state_dict's keys and shapes, in order
  repbn8_golden.npz  4 crops (make_crops seed 31, slots 0..3): logits,
                     checksums + samples of the features2 output and of the
                     GGCA-weighted features, and the folded 3x3 weights of
                     features1.3 (one DEConv) for the host-fold test
"""
from __future__ import annotations

import ast
import json
import sys
from pathlib import Path

sys.dont_write_bytecode = True
REPO = Path(__file__).resolve().parents[1]
REF = Path("/root/reference/CViT-main/model/cvit_GGCA_ADD_DEConv_RepBn8.py")
OUT = REPO / "tests" / "golden"
sys.path.insert(0, str(REPO))

import numpy as np  # noqa: E402
import torch  # noqa: E402
from torch import nn  # noqa: E402

from fac_fake_amd.weights import make_crops, make_repbn8_state_dict  # noqa: E402
from tools.make_golden import ref_normalize  # noqa: E402


def load_reference_namespace():
    tree = ast.parse(REF.read_text(), filename=str(REF))
    keep = []
    for node in tree.body:
        if isinstance(node, (ast.Import, ast.ImportFrom)):
            mods = [a.name for a in node.names] + ([node.module] if isinstance(node, ast.ImportFrom) else [])
            if any(m and m.startswith("torchsummary") for m in mods):
                continue
            keep.append(node)
        elif isinstance(node, (ast.ClassDef, ast.Assign)):
            keep.append(node)
    mod = ast.Module(body=keep, type_ignores=[])
    ns = {"__name__": "repbn8_reference"}
    exec(compile(mod, str(REF), "exec"), ns)
    return ns


def main():
    torch.manual_seed(0)
    torch.cuda.FloatTensor = lambda *shape: torch.empty(*shape, dtype=torch.float32)  # CPU scratch, see above
    nn.Conv1d.cuda = lambda self, *a, **k: self
    ns = load_reference_namespace()
    m = ns["CViT"](image_size=224, patch_size=7, num_classes=2, channels=512, dim=1024, depth=6, heads=8,
                   mlp_dim=2048).eval()
    ref_sd = m.state_dict()
    keys = [[k, list(v.shape)] for k, v in ref_sd.items()]
    (OUT / "repbn8_keys.json").write_text(json.dumps(keys))
    sd = make_repbn8_state_dict(0)
    m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in sd.items()})

    crops = make_crops(4, seed=31)
    x = ref_normalize(crops)
    got = {}
    m.features2.register_forward_hook(lambda mod, i, o: got.__setitem__("f2", o.detach().clone()))
    m.ggca.register_forward_hook(lambda mod, i, o: got.__setitem__("g", o.detach().clone()))
    with torch.no_grad():
        logits = m(x)
        w3, b3 = [], None
        dc = m.features1[3]
        parts = [dc.conv1_1.get_weight(), dc.conv1_2.get_weight(), dc.conv1_3.get_weight(), dc.conv1_4.get_weight(),
                 (dc.conv1_5.weight, dc.conv1_5.bias)]
        w3 = parts[0][0] + parts[1][0] + parts[2][0] + parts[3][0] + parts[4][0]
        b3 = parts[0][1] + parts[1][1] + parts[2][1] + parts[3][1] + parts[4][1]
    f2 = got["f2"].numpy()
    weighted = (got["f2"] * got["g"]).numpy()   # x = x * ggca(x) (:436-437)
    np.savez_compressed(
        OUT / "repbn8_golden.npz",
        crop_seed=np.int64(31), logits=logits.numpy(),
        f2_sum=np.float64(f2.astype(np.float64).sum()), f2_abs=np.float64(np.abs(f2).astype(np.float64).sum()),
        f2_sample=f2.reshape(-1)[::997].copy(),
        weighted_sum=np.float64(weighted.astype(np.float64).sum()), weighted_sample=weighted.reshape(-1)[::997].copy(),
        deconv_w=w3.numpy(), deconv_b=b3.numpy())
    print("logits", logits.numpy())
    print("f2 range", f2.min(), f2.max(), "mean|f2|", np.abs(f2).mean(), "weighted range", weighted.min(),
          weighted.max())


if __name__ == "__main__":
    main()
