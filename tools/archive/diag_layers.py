"""GPU diagnostic: per-layer error of the HIP stem vs the oracle emulation and
vs fp32, plus end-to-end logits.  Run on the GPU box:
    python tools/diag_layers.py [fp16|bf16]
"""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from fac_fake_amd import _lib  # noqa: E402
from fac_fake_amd.cvit import CViT  # noqa: E402
from fac_fake_amd.weights import make_crops, make_state_dict  # noqa: E402
from oracle.cvit_torch import forward_emulated, forward_fp32, normalize_u8  # noqa: E402


def rel(a, b):
    return float((a - b).pow(2).mean().sqrt() / (b.pow(2).mean().sqrt() + 1e-12))


def main(dt):
    torch.set_num_threads(16)
    sd = make_state_dict(0)
    m = CViT(dtype=dt)
    m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in sd.items()})
    m.to("cuda:0")
    crops = make_crops(2, seed=12)
    x = normalize_u8(crops)
    _, fe = forward_emulated(sd, x, dtype=dt, return_features=True)
    _, ff = forward_fp32(sd, x, return_features=True)
    lib = _lib.load()
    xd = torch.from_numpy(crops).cuda()
    m.reserve(8, "cuda:0")
    tdt = torch.float16 if dt == "fp16" else torch.bfloat16
    for layer, (e, f) in enumerate(zip(fe, ff)):
        e = e.permute(0, 2, 3, 1).contiguous()
        f = f.permute(0, 2, 3, 1).contiguous()
        out = torch.empty(e.shape, dtype=tdt, device="cuda:0")
        _lib.check(lib.fac_debug_features_u8(m._ctx, xd.data_ptr(), 2, layer, out.data_ptr(), None), m._ctx, "dbg")
        torch.cuda.synchronize()
        g = out.float().cpu()
        d = (g - e).abs()
        idx = np.unravel_index(int(d.argmax()), d.shape)
        print(f"layer {layer:2d} {tuple(e.shape)} gpu-vs-emu rel {rel(g, e):.3e} max {float(d.max()):.3e} at {idx} "
              f"(emu {float(e[idx]):.4f} gpu {float(g[idx]):.4f})  emu-vs-fp32 rel {rel(e, f):.3e} "
              f"gpu-vs-fp32 rel {rel(g, f):.3e}  frac(!=) {float((g != e).float().mean()):.3e}")
    crops = make_crops(8, seed=11)
    slots = np.array([0, 5, 31, 7, 7, 12, 30, 1])
    x = normalize_u8(crops)
    em = forward_emulated(sd, x, pos_index=slots, dtype=dt)
    fp = forward_fp32(sd, x, pos_index=slots)
    g = m.forward_u8(torch.from_numpy(crops).cuda(), pos_index=slots).cpu()
    print("logits gpu-emu", float((g - em).abs().max()), "emu-fp32", float((em - fp).abs().max()),
          "gpu-fp32", float((g - fp).abs().max()))


if __name__ == "__main__":
    for dt in sys.argv[1:] or ["fp16", "bf16"]:
        print("=====", dt)
        main(dt)
