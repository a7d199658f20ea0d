"""Golden outcomes of the reference CViT's `mask=` argument (cvit.py:50-55).

Imports CViT-main/model/cvit.py (build container only), runs it on random
inputs with masks of several batch sizes and patterns and records, per case,
what the reference does: raise (exception type), return logits equal to the
unmasked forward, or return NaN logits (which rows).  Writes
tests/golden/mask_semantics.json.

    PYTHONDONTWRITEBYTECODE=1 python tools/make_golden_mask.py
"""
import json
import sys
from pathlib import Path

import torch

REF = Path("/root/reference/CViT-main/model")
OUT = Path(__file__).resolve().parents[1] / "tests" / "golden" / "mask_semantics.json"


def main():
    sys.path.insert(0, str(REF))
    from cvit import CViT  # noqa: E402  (the reference module)
    torch.manual_seed(0)
    m = CViT().eval()
    cases = []
    for B in (1, 2, 3, 8, 16):
        x = torch.randn(B, 3, 224, 224)
        for name in ("all_true", "one_false", "all_false", "wide"):
            if name == "wide":
                mask = torch.ones(B, 2, dtype=torch.bool)
            else:
                mask = torch.ones(B, 1, dtype=torch.bool)
                if name == "one_false":
                    mask[B // 2, 0] = False
                if name == "all_false":
                    mask[:] = False
            rec = {"B": B, "pattern": name, "mask": mask.int().tolist()}
            try:
                with torch.no_grad():
                    y, y0 = m(x, mask), m(x)
                rec["outcome"] = "equal" if torch.equal(y, y0) else "nan"
                rec["nan_rows"] = torch.isnan(y).any(1).tolist()
            except Exception as e:  # noqa: BLE001
                rec["outcome"] = "error"
                rec["error"] = type(e).__name__
            cases.append(rec)
    OUT.write_text(json.dumps(cases, indent=1))
    print(f"wrote {OUT} ({len(cases)} cases)")


if __name__ == "__main__":
    main()
