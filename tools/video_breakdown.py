"""Where config 3's dense-mode video time goes (GPU box): host-timed parts of
video.predict_video on the 300-frame 1080x1920 synthetic video.

    python tools/video_breakdown.py
"""
import sys
import time
from pathlib import Path

import numpy as np
import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from fac_fake_amd import video  # noqa: E402
from fac_fake_amd.cvit import CViT  # noqa: E402
from fac_fake_amd.prediction import dense_slots  # noqa: E402
from fac_fake_amd.weights import make_state_dict  # noqa: E402


def timed(f, reps=10):
    f()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        f()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    return float(np.median(ts)) * 1e3


def main():
    dev = torch.device("cuda:0")
    m = CViT(dtype="bf16")
    m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in make_state_dict(0).items()})
    m.to(dev)
    m.reserve(256, dev)
    frames, boxes = video.synthetic_video(300, 1080, 1920, seed=3, device=dev)
    crops = video.crop_faces(frames, boxes)
    slots = torch.from_numpy(dense_slots(300))
    slots_d = slots.to(dev)
    lg = m.forward_u8(crops, pos_index=slots)
    print("crop_faces (incl. box H2D)   %.3f ms" % timed(lambda: video.crop_faces(frames, boxes)))
    print("forward_u8 B=300 host slots  %.3f ms" % timed(lambda: m.forward_u8(crops, pos_index=slots)))
    print("forward_u8 B=300 dev slots   %.3f ms" % timed(lambda: m.forward_u8(crops, pos_index=slots_d)))
    for ch in (160, 100, 64):
        print("pipelined chunk %3d          %.3f ms" % (ch, timed(lambda: m.forward_u8_pipelined(crops, slots_d, chunk=ch))))
    for ch in (256, 224, 192):
        print("pipelined %3d + rest         %.3f ms" % (ch, timed(lambda: m.forward_u8_pipelined(crops, slots_d, chunk=ch,
                                                                                                equal=False))))
    print("forward_u8 B=256             %.3f ms" % timed(lambda: m.forward_u8(crops[:256], pos_index=slots_d[:256])))
    print("device score + item          %.3f ms" % timed(lambda: video.device_video_score(lg)))
    print("predict_video dense          %.3f ms" % timed(lambda: video.predict_video(m, frames, boxes, mode="dense")))


if __name__ == "__main__" and len(sys.argv) == 1:
    main()


def stages():
    import ctypes
    from fac_fake_amd import _lib
    from fac_fake_amd.weights import make_crops
    dev = torch.device("cuda:0")
    m = CViT(dtype="bf16")
    m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in make_state_dict(0).items()})
    m.to(dev)
    m.reserve(320, dev)
    lib = _lib.load()
    names = [f"conv{i + 1}" for i in range(17)] + ["patch_embed", "transformer", "head"]
    for B in (256, 300, 320):
        x = torch.from_numpy(make_crops(B, seed=3)).to(dev)
        p = (torch.arange(B, device=dev) % 32).to(torch.int32)
        lg = torch.empty(B, 2, device=dev)
        st = (ctypes.c_float * 20)()
        acc = np.zeros(20)
        for r in range(4):
            _lib.check(lib.fac_profile_forward_u8(m._ctx, x.data_ptr(), B, p.data_ptr(), lg.data_ptr(), st, 20,
                                                  torch.cuda.current_stream().cuda_stream), m._ctx, "prof")
            if r:
                acc += np.frombuffer(st, dtype=np.float32)
        acc /= 3
        print(B, "total %.3f ms" % acc.sum(), " ".join(f"{n}={v:.3f}" for n, v in zip(names, acc) if v))


if __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "stages":
    stages()
