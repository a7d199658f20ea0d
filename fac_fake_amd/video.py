"""Config 3: one video through face crops -> CViT -> video score, on 1..N GPUs.

The reference's ``predict`` (CViT-main/cvit_prediction.py:153-242) reads
frames with cv2, finds faces with face_recognition (dlib HOG, CPU), crops and
resizes them (``face_face_rec`` :106-121) and scores the crops.  Detection
and video decoding stay outside this path ("only the
crop/resize part is in scope, on synthetic boxes"), so a video here is a
device tensor of decoded BGR frames plus one face box list per frame, and
everything from the crop on runs on the GPU:

* ``crop_faces``: ``frame[top:bottom, left:right]`` -> INTER_AREA resize to
  224x224 -> BGR->RGB, all boxes in one ``fac_crop_resize_u8`` launch
  (fac_fake_amd/csrc/crop.hip), uint8 straight into the conv stack's input
  layout (the reference's float NCHW H2D copy and per-image Python
  normalisation loop, :206-215, disappear: normalisation is fused into conv1).
* ``mode="reference"``: the reference's frame schedule (``frame_indices``:
  frames 0, 0, 5, 10, ... for int(0.1 * length) reads, :165-198), at most
  5 faces per frame (:110) and 29 crops per video (:194), one chunk of slots
  0..n-1; the video score as ``pre_process_prediction(pred_sig(.))``.
* ``mode="dense"``: every box of every frame, crop j at pos slot j mod 32,
  sharded contiguously over the ranks of ``group`` (one process per GPU); the
  only collective is the all-gather of per-crop logits (``sharding``,
  RCCL over xGMI with backend "nccl") before the score.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.distributed as dist

from . import _lib
from .prediction import EMPTY_SCORE, chunk_slots, dense_slots
from .sharding import gather_logits, shard_bounds
from .weights import splitmix64

CROP = 224
FACES_PER_FRAME = 5          # cvit_prediction.py:110 (count < 5)
MAX_CROPS_REFERENCE = 29     # cvit_prediction.py:194 (count_face_rec < 29)
FRAME_JUMP = 5               # cvit_prediction.py:168


def frame_indices(length: int) -> list[int]:
    """Frames the reference reads: int(0.1 * length) iterations of read-then-seek
    (cvit_prediction.py:165-198), i.e. 0, 0, 5, 10, ... (every read successful)."""
    count = int(length * 0.1)
    out, pos, start = [], 0, 0
    for _ in range(count):
        out.append(pos)
        pos, start = start, start + FRAME_JUMP
    return out


BOX_MIN, BOX_SPAN = 112, 448   # synthetic face boxes: square, 112..559 px


def synthetic_video(n_frames: int, height: int = 1080, width: int = 1920, seed: int = 3, device=None,
                    faces_per_frame: int = 1, box_min: int = BOX_MIN, box_span: int = BOX_SPAN):
    """Deterministic synthetic video: uint8 BGR frames [F, H, W, 3] on `device`
    (torch's seeded device generator) and face boxes int32 [F*k, 5] =
    (frame, left, top, right, bottom), square boxes of box_min..box_min +
    box_span - 1 px inside the frame (splitmix64 of `seed`).  The default
    112..559 puts about a quarter of them under 224 px, so both of cv2's
    INTER_AREA branches (area average / upscale) are exercised; round 1's
    config-3 numbers used 240..559 (box_min=240, box_span=320), where every
    crop is an area-average downscale."""
    dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
    g = torch.Generator(device=dev).manual_seed(seed)
    frames = torch.randint(0, 256, (n_frames, height, width, 3), dtype=torch.uint8, device=dev, generator=g)
    r = splitmix64(np.arange(3 * n_frames * faces_per_frame, dtype=np.uint64), seed + 1000).reshape(-1, 3)
    size = box_min + (r[:, 0] % np.uint64(box_span)).astype(np.int64)
    size = np.minimum(size, min(height, width))
    left = (r[:, 1] % (np.uint64(width) - size.astype(np.uint64) + np.uint64(1))).astype(np.int64)
    top = (r[:, 2] % (np.uint64(height) - size.astype(np.uint64) + np.uint64(1))).astype(np.int64)
    f = np.repeat(np.arange(n_frames, dtype=np.int64), faces_per_frame)
    boxes = np.stack([f, left, top, left + size, top + size], 1).astype(np.int32)
    return frames, boxes


def crop_faces(frames: torch.Tensor, boxes, out: torch.Tensor | None = None) -> torch.Tensor:
    """uint8 BGR frames [F, H, W, 3] (device) + boxes [n, 5] -> uint8 RGB crops
    [n, 224, 224, 3] (device; written into ``out`` when given, a contiguous
    [n, 224, 224, 3] uint8 tensor on the frames' device)."""
    if not frames.is_cuda or frames.dtype != torch.uint8 or frames.dim() != 4 or frames.shape[3] != 3:
        raise ValueError("frames must be a uint8 [F, H, W, 3] device tensor")
    b = torch.as_tensor(np.asarray(boxes, dtype=np.int32).reshape(-1, 5)).to(frames.device)
    n = int(b.shape[0])
    if out is None:
        crops = torch.empty(n, CROP, CROP, 3, dtype=torch.uint8, device=frames.device)
    else:
        if (out.dtype != torch.uint8 or tuple(out.shape) != (n, CROP, CROP, 3) or not out.is_contiguous()
                or out.device != frames.device):
            raise ValueError(f"out must be a contiguous uint8 [{n},{CROP},{CROP},3] tensor on {frames.device}")
        crops = out
    if n:
        frames = frames.contiguous()
        F, H, W, _ = frames.shape
        lib = _lib.load()
        _lib.check(lib.fac_crop_resize_u8(frames.data_ptr(), F, H, W, b.data_ptr(), n, crops.data_ptr(),
                                          torch.cuda.current_stream(frames.device).cuda_stream),
                   None, "fac_crop_resize_u8")
    return crops


def reference_boxes(boxes, length: int) -> np.ndarray:
    """The boxes the reference would crop: per frame read (frame_indices), that
    frame's first 5 faces, until 29 crops (cvit_prediction.py:107-121,189-196)."""
    boxes = np.asarray(boxes, dtype=np.int32).reshape(-1, 5)
    # each frame's first FACES_PER_FRAME boxes, in list order (a stable sort
    # by frame keeps it), located by binary search per frame read
    order = np.argsort(boxes[:, 0], kind="stable")
    by_frame = boxes[order]
    fi = np.asarray(frame_indices(length), dtype=np.int64)
    lo = np.searchsorted(by_frame[:, 0], fi, "left")
    cnt = np.minimum(np.searchsorted(by_frame[:, 0], fi, "right") - lo, FACES_PER_FRAME)
    start = np.repeat(lo - (np.cumsum(cnt) - cnt), cnt)   # row of the k-th crop = its read's lo + rank
    idx = (start + np.arange(int(cnt.sum())))[:MAX_CROPS_REFERENCE]
    return by_frame[idx].astype(np.int32).reshape(-1, 5)


def predict_video(model, frames: torch.Tensor, boxes, mode: str = "reference", group=None,
                  return_logits: bool = False):
    """Video probability (< 0.5 REAL, >= 0.5 FAKE) of one video.

    ``model``: fac_fake_amd.cvit.CViT (weights loaded, on this rank's GPU);
    ``frames``: the decoded video, a device tensor or (dense mode) a host
    array / CPU tensor, of which each rank then uploads only the frames of
    its own shard of crops; ``boxes``: [n, 5] (frame, left, top, right,
    bottom).  In dense mode with a process group, every rank must call this
    with the same ``boxes``.
    """
    if mode == "reference":
        fr, sel = select_reference(frames, boxes)
        if len(sel) == 0:
            return (float(EMPTY_SCORE), None) if return_logits else float(EMPTY_SCORE)
        if not (isinstance(fr, torch.Tensor) and fr.is_cuda):
            fr = torch.as_tensor(np.ascontiguousarray(fr)).to(_work_device(frames))
        crops = crop_faces(fr, sel)
        # <= 29 crops: one chunk, slots 0..n-1 = the model's default slots
        # (cached on the device: no host->device copy per video)
        slots = None if len(sel) <= 32 else torch.from_numpy(chunk_slots(len(sel)))
        with torch.no_grad():
            logits = model.forward_u8(crops, pos_index=slots)
    elif mode == "dense":
        boxes = np.asarray(boxes, dtype=np.int32).reshape(-1, 5)
        n = len(boxes)
        if n == 0:
            return (float(EMPTY_SCORE), None) if return_logits else float(EMPTY_SCORE)
        world = dist.get_world_size(group) if group is not None or dist.is_initialized() else 1
        rank = dist.get_rank(group) if world > 1 else 0
        lo, hi = shard_bounds(n, world, rank)
        dev = _work_device(frames)
        if hi > lo:
            fr, sel = frames, boxes[lo:hi]
            if not (isinstance(frames, torch.Tensor) and frames.is_cuda):
                # a host video: this rank uploads only the frames of its own
                # crops (a contiguous shard), not the whole decoded video
                ids, inv = np.unique(sel[:, 0], return_inverse=True)
                fr = torch.as_tensor(np.ascontiguousarray(np.asarray(frames)[ids.astype(np.int64)])).to(dev)
                sel = sel.copy()
                sel[:, 0] = inv.reshape(-1).astype(np.int32)
            crops = crop_faces(fr, sel)
            # one forward over the rank's crops: splitting them into pipelined
            # chunks (CViT.forward_u8_pipelined) measured slower for a 300-crop
            # video (4.73-5.13 vs 4.55 ms: two half batches fill the GPU worse
            # than their overlap saves; tools/video_breakdown.py)
            with torch.no_grad():
                local = model.forward_u8(crops, pos_index=torch.from_numpy(dense_slots(hi - lo, offset=lo)))
        else:
            local = torch.zeros(0, 2, dtype=torch.float32, device=dev)
        logits = gather_logits(local.float(), n, group) if world > 1 else local
    else:
        raise ValueError("mode must be 'reference' or 'dense'")
    score = device_video_score(logits)
    return (score, logits) if return_logits else score


def _work_device(frames) -> torch.device:
    """Where a video's crops are made: the frames' GPU, else the current GPU
    (host frames are uploaded there); a CPU-only process keeps host frames on
    the CPU (the model call then fails loudly: there is no CPU path)."""
    if isinstance(frames, torch.Tensor) and frames.is_cuda:
        return frames.device
    return torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu")


def select_reference(frames, boxes):
    """The reference's crop selection for one video (``reference_boxes``) and
    the frames it needs: ``(frames, sel)`` with ``sel`` [n, 5] indexing into
    the returned frames.  A device tensor is returned as is; a host video
    (numpy array / CPU tensor) is cut down to the frames the schedule reads
    (int(0.1 * F) reads, :165-198: ~30 frames of a 300-frame 1080p video,
    187 MB instead of 1.87 GB to hold and to upload)."""
    sel = reference_boxes(boxes, int(frames.shape[0]))
    if isinstance(frames, torch.Tensor) and frames.is_cuda:
        return frames, sel
    ids, inv = np.unique(sel[:, 0], return_inverse=True)
    sub = np.asarray(frames)[ids.astype(np.int64)] if len(sel) else np.zeros((0, 1, 1, 3), np.uint8)
    sel = sel.copy()
    sel[:, 0] = inv.reshape(-1).astype(np.int32)
    return sub, sel


def score_selected(model, items, batch: int = 256, device=None, return_logits: bool = False):
    """Reference-mode scores of videos whose crops are already selected:
    ``items`` = [(frames, sel)] as ``select_reference`` returns them.  Each
    video keeps its own chunk slots 0..n-1 (``chunk_slots``); the crops of
    all videos are concatenated, scored in forwards of at most ``batch``
    crops (pipelined: batch k's encoder beside batch k+1's conv stack), and
    reduced per video by one ``fac_video_score_seg`` launch."""
    items = list(items)
    if not items:
        return ([], None) if return_logits else []
    dev = torch.device(device) if device is not None else None
    if dev is None:
        for fr, _ in items:
            if isinstance(fr, torch.Tensor) and fr.is_cuda:
                dev = fr.device
                break
        else:
            dev = torch.device("cuda", torch.cuda.current_device())
    seg = np.zeros(len(items) + 1, dtype=np.int32)
    np.cumsum([len(sel) for _, sel in items], out=seg[1:])
    total = int(seg[-1])
    crops = torch.empty(total, CROP, CROP, 3, dtype=torch.uint8, device=dev)
    pos = np.zeros(total, dtype=np.int32)
    for v, (frames, sel) in enumerate(items):
        if len(sel) == 0:
            continue
        fr = frames if isinstance(frames, torch.Tensor) and frames.is_cuda else \
            torch.as_tensor(np.ascontiguousarray(frames)).to(dev)
        crop_faces(fr, sel, out=crops[seg[v]:seg[v + 1]])
        pos[seg[v]:seg[v + 1]] = chunk_slots(len(sel))
    with torch.no_grad():
        if total == 0:
            logits = torch.zeros(0, 2, dtype=torch.float32, device=dev)
        elif total <= batch:
            logits = model.forward_u8(crops, pos_index=torch.from_numpy(pos))
        else:
            logits = model.forward_u8_pipelined(crops, torch.from_numpy(pos), chunk=batch, equal=False)
    scores = segmented_video_scores(logits, seg)
    return (scores, logits) if return_logits else scores


def predict_videos(model, videos, batch: int = 256, device=None, return_logits: bool = False):
    """Reference-mode scores of several videos (cvit_prediction.py:73-83 runs
    ``predict`` video after video, one <= 29-crop forward each), with the
    crops of many videos in one forward.

    ``videos``: iterable of ``(frames, boxes)``: decoded BGR uint8 frames
    [F, H, W, 3] (device tensor, or host array / CPU tensor: only the frames
    the schedule reads are uploaded) and boxes [n, 5] (frame, left, top,
    right, bottom).  A crop's logits do not depend on its batch (fixed
    split-K orders, no cross-crop op before the score) and the segmented
    score sums each video's sigmoids in crop order, so every score is
    bit-identical to ``predict_video(model, frames, boxes)``.  Returns a list
    of floats (and the [N, 2] logits with ``return_logits``).
    """
    return score_selected(model, [select_reference(f, b) for f, b in videos], batch, device, return_logits)


def segmented_video_scores(logits: torch.Tensor, seg) -> list:
    """Per-video ``pre_process_prediction(pred_sig(.))`` of logit rows
    [seg[v], seg[v+1]) (fac_video_score_seg), one device->host read."""
    seg = np.asarray(seg, dtype=np.int32)
    nv = len(seg) - 1
    if nv <= 0:
        return []
    if int(seg[-1]) == 0:   # no crop in any of these videos: each scores 0.5 (cvit_prediction.py:218-219)
        return [float(EMPTY_SCORE)] * nv
    logits = logits.float().contiguous()
    d_seg = torch.from_numpy(seg).to(logits.device)
    out = torch.empty(nv, dtype=torch.float32, device=logits.device)
    _lib.check(_lib.load().fac_video_score_seg(logits.data_ptr(), d_seg.data_ptr(), nv, out.data_ptr(),
                                               torch.cuda.current_stream(logits.device).cuda_stream),
               None, "fac_video_score_seg")
    return [float(s) for s in out.cpu().tolist()]


def device_video_score(logits: torch.Tensor) -> float:
    """pre_process_prediction(pred_sig(logits)) (cvit_prediction.py:240,
    258-281) on the GPU (fac_video_score: per-logit sigmoid, fp32 column sums
    in crop order, the f > r rule), then the one device->host read the
    reference makes (.item(), :242)."""
    logits = logits.float().contiguous()
    out = torch.empty((), dtype=torch.float32, device=logits.device)
    _lib.check(_lib.load().fac_video_score(logits.data_ptr(), int(logits.shape[0]), out.data_ptr(),
                                           torch.cuda.current_stream(logits.device).cuda_stream),
               None, "fac_video_score")
    return float(out.item())
