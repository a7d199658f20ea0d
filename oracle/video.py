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
* cv2 computes true area averages only when BOTH axes shrink or keep their
  size (a box of at least 224 px on each side).  Otherwise -- a face box under
  224 px on either axis, common on 480p/720p footage -- ``cv2.resize`` runs
  its bilinear path with area-mode coefficients on both axes
  (``linear_area_coeffs``: source index floor(d*scale), fraction
  (d+1) - (s+1)/scale wrapped to [0,1), 11-bit fixed-point taps), a
  horizontal pass in exact integers and the vertical pass of its SIMD kernel
  for uint8 (``VResizeLinearVec_32s8u``: rows >> 4, 16-bit mulhi with the row
  taps, (sum + 2) >> 2, saturate).  ``crop_resize_area`` takes that branch
  whenever the clipped box is under 224 px on either axis.  This restates
  OpenCV's published algorithm (opencv/modules/imgproc/src/resize.cpp,
  ``hal::resize`` / ``resizeGeneric_`` / ``HResizeLinear`` /
  ``VResizeLinearVec_32s8u``, OpenCV 4.x, 128/256-bit SIMD builds); the
  reference pins no OpenCV version and cv2 is not in the image, so parity
  with cv2 on these boxes is unpinned (non-SIMD builds round the vertical
  pass as (b0 D0 + b1 D1 + 2^21) >> 22 and can differ by one count).
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


def linear_area_coeffs(n: int, clamp_fraction: bool):
    """cv2's INTER_AREA coefficients on a non-downscale (hal::resize's
    ``area_mode`` branch of the x and y coefficient loops), n source pixels ->
    224: per output pixel d, the first source index s and the fixed-point
    taps (a0, a1) of s and s + 1 in units of 1/2048.  ``clamp_fraction``: the
    x loop also pins s = n - 1 with fraction 0 once s + 1 leaves the span
    (the y loop leaves the fraction alone and clips the row indices)."""
    inv = CROP / n           # inv_scale = (double)dsize / ssize
    scale = 1.0 / inv        # scale = 1. / inv_scale
    s_out = np.empty(CROP, np.int64)
    taps = np.empty((CROP, 2), np.int64)
    for d in range(CROP):
        s = int(np.floor(d * scale))
        f = np.float32((d + 1) - (s + 1) * inv)            # (float)((d+1) - (s+1)*inv_scale), double math
        f = np.float32(0.0) if f <= 0 else np.float32(f - np.float32(np.floor(f)))
        if clamp_fraction and s >= n - 1:
            s, f = n - 1, np.float32(0.0)
        s_out[d] = s
        c0, c1 = np.float32(np.float32(1.0) - f), f
        taps[d] = (int(np.rint(np.float32(c0 * np.float32(2048)))),
                   int(np.rint(np.float32(c1 * np.float32(2048)))))  # saturate_cast<short>: round half even
    return s_out, taps


def _resize_linear_area(src: np.ndarray) -> np.ndarray:
    """src int64 [ny, nx, 3] (box, BGR) -> uint8 [224, 224, 3] BGR, cv2's
    bilinear-with-area-coefficients path (see the module docstring)."""
    ny, nx = src.shape[:2]
    sx, ax = linear_area_coeffs(nx, True)
    sy, by = linear_area_coeffs(ny, False)
    sx1 = np.minimum(sx + 1, nx - 1)   # a1 == 0 wherever the second tap is clamped
    # horizontal pass, exact integers: D[row, d, c] = S[row, sx] a0 + S[row, sx+1] a1
    D = src[:, sx, :] * ax[None, :, 0, None] + src[:, sx1, :] * ax[None, :, 1, None]
    r0 = np.clip(sy, 0, ny - 1)
    r1 = np.clip(sy + 1, 0, ny - 1)
    h0 = np.minimum(D[r0] >> 4, 32767)            # v_pack(v_shr<4>(S)) (saturating to int16)
    h1 = np.minimum(D[r1] >> 4, 32767)
    v = ((h0 * by[:, 0, None, None]) >> 16) + ((h1 * by[:, 1, None, None]) >> 16)   # v_mul_hi
    return np.clip((v + 2) >> 2, 0, 255).astype(np.uint8)                          # v_rshr_pack_u<2>


def crop_resize_area(frame: np.ndarray, box) -> np.ndarray:
    """frame: uint8 [H, W, 3] BGR; box = (left, top, right, bottom) -> uint8 [224, 224, 3] RGB."""
    H, W = frame.shape[:2]
    left, top, right, bottom = (int(v) for v in box)
    x0, y0, x1, y1 = max(left, 0), max(top, 0), min(right, W), min(bottom, H)
    if x1 <= x0 or y1 <= y0:
        return np.zeros((CROP, CROP, 3), np.uint8)
    src = frame[y0:y1, x0:x1].astype(np.int64)
    if (x1 - x0) < CROP or (y1 - y0) < CROP:
        return np.ascontiguousarray(_resize_linear_area(src)[:, :, ::-1])  # BGR -> RGB
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
