"""Config-3 video preprocessing, restated on the CPU (numpy).

TEST INFRASTRUCTURE ONLY (the checker, never the product path).

* ``reference_frame_indices(length)`` restates the frame schedule of
  ``cvit_prediction.py:165-198``: ``frame_count = int(length * 0.1)`` loop
  iterations, each doing ``cap.read()`` (the frame at the current position)
  then ``cap.set(CAP_PROP_POS_FRAMES, start)`` with ``start`` = 0, 5, 10, ...
  advanced after every successful read, so the frames read are
  0, 0, 5, 10, ..., 5 * (frame_count - 2).  At most 29 crops are kept
  (``:191-196``).
* ``crop_resize_area(frame, box)`` restates ``frame[top:bottom, left:right]``
  -> ``cv2.resize(.., (224, 224), INTER_AREA)`` -> ``cv2.cvtColor(RGB2BGR)``
  (``:111-116``).  INTER_AREA's area weights are evaluated exactly in integer
  arithmetic: output pixel o of an n-pixel span covers [o*n, (o+1)*n) in
  units of 1/224 pixel, source pixel s covers [224 s, 224 s + 224), the
  weight is the integer overlap, and out = round-half-up(sum / (n_x n_y)).
  The HIP kernel (fac_fake_amd/csrc/crop.hip) evaluates the same integers.
  cv2 is absent from the image, so agreement with cv2 itself (float weights,
  possible 1-count differences on exact .5 ties) is unpinned.
"""
from __future__ import annotations

import numpy as np

CROP = 224
MAX_CROPS_REFERENCE = 29  # cvit_prediction.py:194 (count_face_rec < 29)


def reference_frame_indices(length: int, frame_jump: int = 5) -> list[int]:
    """Frames the reference's ``predict`` reads from a ``length``-frame video
    (cvit_prediction.py:163-198; every read assumed successful)."""
    frame_count = int(length * 0.1)
    pos, start, out = 0, 0, []
    for _ in range(frame_count):
        out.append(pos)          # cap.read() returns the frame at the current position
        pos = start              # cap.set(CAP_PROP_POS_FRAMES, start_frame_number)
        start += frame_jump      # start_frame_number += frame_jump (after a successful read)
    return out


def overlap_matrix(n: int) -> np.ndarray:
    """R[o, s] = overlap (in 1/224 px) of output pixel o's interval with source pixel s."""
    o = np.arange(CROP, dtype=np.int64)[:, None]
    s = np.arange(n, dtype=np.int64)[None, :]
    lo = np.maximum(o * n, s * CROP)
    hi = np.minimum((o + 1) * n, (s + 1) * CROP)
    return np.maximum(hi - lo, 0)


def crop_resize_area(frame: np.ndarray, box) -> np.ndarray:
    """frame: uint8 [H, W, 3] BGR; box = (left, top, right, bottom) -> uint8 [224, 224, 3] RGB."""
    H, W = frame.shape[:2]
    left, top, right, bottom = (int(v) for v in box)
    x0, y0, x1, y1 = max(left, 0), max(top, 0), min(right, W), min(bottom, H)
    if x1 <= x0 or y1 <= y0:
        return np.zeros((CROP, CROP, 3), np.uint8)
    src = frame[y0:y1, x0:x1].astype(np.int64)
    ry, rx = overlap_matrix(y1 - y0), overlap_matrix(x1 - x0)
    den = (x1 - x0) * (y1 - y0)
    out = np.empty((CROP, CROP, 3), np.uint8)
    for c in range(3):
        num = ry @ src[:, :, c] @ rx.T
        out[:, :, 2 - c] = ((2 * num + den) // (2 * den)).astype(np.uint8)  # BGR -> RGB
    return out


def crop_batch(frames: np.ndarray, boxes: np.ndarray) -> np.ndarray:
    """frames uint8 [F, H, W, 3]; boxes int [n, 5] = (frame, left, top, right, bottom)."""
    out = np.zeros((len(boxes), CROP, CROP, 3), np.uint8)
    for i, (f, l, t, r, b) in enumerate(np.asarray(boxes)):
        if 0 <= f < len(frames):
            out[i] = crop_resize_area(frames[f], (l, t, r, b))
    return out
