"""Where config 3's reference-mode call goes (GPU box): the reference scores a
video as ONE forward of <= 29 crops (cvit_prediction.py:224-229).  Host-timed
pieces of video.predict_video(mode="reference") on the 300-frame 1080x1920
synthetic video, the B = 29 forward with and without the small-batch graph,
and the per-stage GPU times of one B = 29 forward.

    python tools/ref_latency.py [--dtype bf16]
"""
import argparse
import ctypes
import sys
import time
from pathlib import Path

import numpy as np
import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from fac_fake_amd import _lib, video  # noqa: E402
from fac_fake_amd.cvit import CViT  # noqa: E402
from fac_fake_amd.weights import make_state_dict  # noqa: E402

NAMES = [f"conv{i + 1}" for i in range(17)] + ["patch_embed", "transformer", "head"]


def timed(f, reps=100):
    for _ in range(10):
        f()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        f()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    return float(np.median(ts)) * 1e3


def device_ms(f, reps=100):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    f()
    torch.cuda.synchronize()
    s.record()
    for _ in range(reps):
        f()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dtype", default="bf16")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    m = CViT(dtype=args.dtype)
    m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in make_state_dict(0).items()})
    m.to(dev)
    m.reserve(256, dev)
    frames, boxes = video.synthetic_video(300, 1080, 1920, seed=3, device=dev)
    fr, sel = video.select_reference(frames, boxes)
    n = len(sel)
    crops = video.crop_faces(fr, sel)
    lg = m.forward_u8(crops)
    for _ in range(300):  # clocks ramp up over ~0.1 s of work
        m.forward_u8(crops)
    torch.cuda.synchronize()
    out = {}
    out["select_reference (host)"] = timed(lambda: video.select_reference(frames, boxes))
    out["crop_faces"] = timed(lambda: video.crop_faces(fr, sel))
    out[f"forward_u8 B={n} graph (host-timed)"] = timed(lambda: m.forward_u8(crops))
    out[f"forward_u8 B={n} graph (device, back-to-back)"] = device_ms(lambda: m.forward_u8(crops))
    m.set_option("graph_max_b", 0)
    out[f"forward_u8 B={n} eager (host-timed)"] = timed(lambda: m.forward_u8(crops))
    out[f"forward_u8 B={n} eager (device, back-to-back)"] = device_ms(lambda: m.forward_u8(crops))
    m.set_option("graph_max_b", 32)
    for gs in (-1, 4, 5, 6):
        for cs in (0, 1):
            m.set_option("gemm_small", gs)
            m.set_option("conv_small", cs)
            out[f"forward_u8 B={n} graph, gemm_small {gs:2d} conv_small {cs} (device)"] = device_ms(
                lambda: m.forward_u8(crops))
    m.set_option("gemm_small", 5)
    m.set_option("conv_small", 1)
    out["device score + item"] = timed(lambda: video.device_video_score(lg))
    out["predict_video reference"] = timed(lambda: video.predict_video(m, frames, boxes, mode="reference"))
    for k, v in out.items():
        print(f"{k:48s} {v:8.3f} ms")
    lib = _lib.load()
    p = torch.arange(n, device=dev, dtype=torch.int32)
    lgb = torch.empty(n, 2, device=dev)
    st = (ctypes.c_float * 20)()
    acc = np.zeros(20)
    reps = 5
    for r in range(reps + 1):
        _lib.check(lib.fac_profile_forward_u8(m._ctx, crops.data_ptr(), n, p.data_ptr(), lgb.data_ptr(), st, 20,
                                              torch.cuda.current_stream().cuda_stream), m._ctx, "prof")
        if r:
            acc += np.frombuffer(st, dtype=np.float32)
    acc /= reps
    print(f"per-stage GPU ms at B={n} (sum {acc.sum():.3f}):")
    print("  " + "  ".join(f"{a}={b:.4f}" for a, b in zip(NAMES, acc)))


if __name__ == "__main__":
    main()
