"""Config 3 (one video: face crops -> CViT -> score) host logic on the CPU.

* the reference's frame schedule and crop caps (cvit_prediction.py:165-198);
* the CPU restatement of crop + INTER_AREA resize + BGR->RGB
  (oracle/video.py) on cases with a closed form: identity at 224, exact box
  averages at integer scales, constants, clipping;
* dense-mode sharding over a 2-rank gloo group: every rank crops and scores
  its contiguous shard, one all-gather, the same logits and score as 1 rank
  (with the oracle's crop and a CPU stand-in scorer: the HIP crop kernel and
  forward are checked against these on the GPU in test_gpu_parity.py).
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from fac_fake_amd import video
from oracle import video as ov


@pytest.mark.parametrize("length", [0, 1, 9, 10, 11, 25, 90, 300, 301])
def test_frame_schedule_matches_restatement(length):
    assert video.frame_indices(length) == ov.reference_frame_indices(length)


def test_frame_schedule_300():
    idx = video.frame_indices(300)
    assert len(idx) == 30 and idx[:4] == [0, 0, 5, 10] and idx[-1] == 140


def test_reference_boxes_caps():
    # 3 faces on every frame: 30 reads x 3 faces, capped at 29 crops; frame 0 read twice
    boxes = np.array([[f, 10 * k, 0, 10 * k + 300, 300] for f in range(300) for k in range(3)], np.int32)
    sel = video.reference_boxes(boxes, 300)
    assert sel.shape == (29, 5)
    assert list(sel[:6, 0]) == [0, 0, 0, 0, 0, 0]
    assert list(sel[6:9, 0]) == [5, 5, 5]
    # 7 faces on one frame: only 5 are taken per read
    boxes = np.array([[0, k, 0, k + 300, 300] for k in range(7)], np.int32)
    assert len(video.reference_boxes(boxes, 10)) == 5


def test_area_resize_identity_at_224():
    rng = np.random.default_rng(0)
    frame = rng.integers(0, 256, (300, 400, 3), dtype=np.uint8)
    out = ov.crop_resize_area(frame, (17, 33, 17 + 224, 33 + 224))
    assert np.array_equal(out, frame[33:257, 17:241, ::-1])


@pytest.mark.parametrize("k", [2, 3])
def test_area_resize_integer_scale_is_box_average(k):
    rng = np.random.default_rng(k)
    frame = rng.integers(0, 256, (224 * k + 5, 224 * k + 9, 3), dtype=np.uint8)
    out = ov.crop_resize_area(frame, (4, 2, 4 + 224 * k, 2 + 224 * k))
    blk = frame[2:2 + 224 * k, 4:4 + 224 * k].astype(np.int64).reshape(224, k, 224, k, 3).sum((1, 3))
    exp = (2 * blk + k * k) // (2 * k * k)
    assert np.array_equal(out, exp[:, :, ::-1].astype(np.uint8))


def test_area_resize_constant_and_clipping():
    frame = np.zeros((500, 600, 3), np.uint8)
    frame[..., 0], frame[..., 1], frame[..., 2] = 10, 20, 30
    out = ov.crop_resize_area(frame, (-50, 100, 333, 577))   # clipped to (0,100,333,500)
    assert (out[..., 0] == 30).all() and (out[..., 1] == 20).all() and (out[..., 2] == 10).all()
    assert not ov.crop_resize_area(frame, (700, 0, 800, 100)).any()  # fully outside: zeros


def test_synthetic_video_is_deterministic_and_in_frame():
    f1, b1 = video.synthetic_video(4, 300, 500, seed=5, device="cpu")
    f2, b2 = video.synthetic_video(4, 300, 500, seed=5, device="cpu")
    assert torch.equal(f1, f2) and np.array_equal(b1, b2)
    assert (b1[:, 1] >= 0).all() and (b1[:, 3] <= 500).all() and (b1[:, 2] >= 0).all() and (b1[:, 4] <= 300).all()
    assert ((b1[:, 3] - b1[:, 1]) >= 112).all()
    _, b3 = video.synthetic_video(1, 1080, 1920, seed=3, device="cpu", faces_per_frame=64)
    side = b3[:, 3] - b3[:, 1]
    assert (side < 224).any() and (side >= 224).any()   # both INTER_AREA branches occur


def _linear_area_scalar(frame, box):
    """Independent scalar loop over cv2's bilinear-with-area-coefficients
    resize for uint8 (resize.cpp: coefficient loops of hal::resize,
    HResizeLinear, VResizeLinearVec_32s8u), used to check the vectorised
    restatement in oracle/video.py."""
    import math
    x0, y0, x1, y1 = box
    src = frame[y0:y1, x0:x1].astype(np.int64)
    ny, nx = src.shape[:2]

    def coeffs(n, d, clamp):
        inv = 224 / n
        scale = 1.0 / inv
        s = math.floor(d * scale)
        f = np.float32((d + 1) - (s + 1) * inv)
        f = np.float32(0) if f <= 0 else np.float32(f - np.float32(math.floor(f)))
        if clamp and s >= n - 1:
            s, f = n - 1, np.float32(0)
        a0 = int(np.rint(np.float32((np.float32(1) - f) * np.float32(2048))))
        a1 = int(np.rint(np.float32(f * np.float32(2048))))
        return s, a0, a1

    out = np.zeros((224, 224, 3), np.uint8)
    for dy in range(224):
        sy, b0, b1 = coeffs(ny, dy, False)
        rows = (min(sy, ny - 1), min(sy + 1, ny - 1))
        for dx in range(224):
            sx, a0, a1 = coeffs(nx, dx, True)
            for c in range(3):
                h = [min((src[r, sx, c] * a0 + src[r, min(sx + 1, nx - 1), c] * a1) >> 4, 32767) for r in rows]
                v = ((h[0] * b0) >> 16) + ((h[1] * b1) >> 16)
                out[dy, dx, 2 - c] = min(max((v + 2) >> 2, 0), 255)
    return out


@pytest.mark.parametrize("k", [2, 4, 8])   # power-of-two factors: scale and 1/scale are exact doubles
def test_area_resize_integer_upscale_replicates_pixels(k):
    """cv2 INTER_AREA enlarging by an integer factor: the area-mode
    fractions are all 0, so every source pixel is repeated k x k times."""
    n = 224 // k
    rng = np.random.default_rng(k)
    frame = rng.integers(0, 256, (n + 10, n + 12, 3), dtype=np.uint8)
    out = ov.crop_resize_area(frame, (3, 5, 3 + n, 5 + n))
    exp = np.repeat(np.repeat(frame[5:5 + n, 3:3 + n], k, 0), k, 1)[:, :, ::-1]
    assert np.array_equal(out, exp)


@pytest.mark.parametrize("box", [(3, 4, 103, 104),      # 100 x 100: both axes enlarge
                                 (0, 0, 300, 150),      # x shrinks, y enlarges (mixed)
                                 (10, 2, 160, 402),     # x enlarges, y shrinks (mixed)
                                 (5, 7, 228, 230),      # 223 x 223
                                 (1, 1, 2, 2),          # one pixel
                                 (0, 0, 224, 131)])     # x identity, y enlarges
def test_linear_area_branch_matches_scalar_restatement(box):
    rng = np.random.default_rng(sum(box))
    frame = rng.integers(0, 256, (420, 320, 3), dtype=np.uint8)
    got = ov.crop_resize_area(frame, box)
    assert np.array_equal(got, _linear_area_scalar(frame, box))


def test_linear_area_branch_constant_and_identity_axis():
    frame = np.full((200, 300, 3), 200, np.uint8)
    frame[..., 1] = 7
    out = ov.crop_resize_area(frame, (0, 0, 150, 90))
    assert (np.abs(out.astype(int) - frame[0, 0, ::-1].astype(int)) <= 1).all()
    rng = np.random.default_rng(1)
    frame = rng.integers(0, 256, (120, 224, 3), dtype=np.uint8)
    out = ov.crop_resize_area(frame, (0, 0, 224, 112))   # x keeps its size, y doubles
    assert np.array_equal(out, np.repeat(frame[:112], 2, 0)[:, :, ::-1])


class _StandInModel:
    """CPU stand-in scorer for the sharding test: logit = f(crop mean, slot)."""

    def forward_u8(self, crops, pos_index):
        m = crops.float().mean((1, 2, 3))
        p = pos_index.float().to(m.device)
        return torch.stack([m / 255.0 - 0.5 + 0.01 * p, 0.5 - m / 255.0], 1)


def _dense_worker(rank, world, port, frames, boxes, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import fac_fake_amd.video as v
        v.crop_faces = lambda fr, bx: torch.from_numpy(ov.crop_batch(fr.numpy(), bx))  # CPU stand-in
        from fac_fake_amd.prediction import pre_process_prediction, pred_sig
        v.device_video_score = lambda lg: float(pre_process_prediction(pred_sig(lg)))  # CPU stand-in
        score, logits = v.predict_video(_StandInModel(), frames, boxes, mode="dense", return_logits=True)
        q.put((rank, score, logits.numpy()))
    finally:
        dist.destroy_process_group()


def test_dense_mode_sharded_over_two_ranks_matches_one():
    frames, boxes = video.synthetic_video(7, 260, 300, seed=9, device="cpu", faces_per_frame=2)
    ref_crops = torch.from_numpy(ov.crop_batch(frames.numpy(), boxes))
    from fac_fake_amd.prediction import dense_slots, pre_process_prediction, pred_sig
    ref_logits = _StandInModel().forward_u8(ref_crops, torch.from_numpy(dense_slots(len(boxes))))
    ref_score = float(pre_process_prediction(pred_sig(ref_logits)))
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    procs = [ctx.Process(target=_dense_worker, args=(r, 2, port, frames, boxes, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    for rank, score, logits in res:
        assert np.array_equal(logits, ref_logits.numpy()), rank
        assert score == ref_score
