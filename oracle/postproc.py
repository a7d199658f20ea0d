"""ORACLE (test infrastructure only): plain-Python restatement of the video
scoring in CViT-main/cvit_prediction.py, used to check fac_fake_amd.prediction
and the device ``video_score`` kernel.

* pred_sig (:258-259): per-logit sigmoid of the squeezed [N,2] logits.
* pre_process_prediction (:266-281): if len > 2 -> f = mean(col0),
  r = mean(col1) as running fp32 sums in order; f if f > r else |1 - r|;
  otherwise 0.5 (so 1 and 2 crops both score 0.5).
* zero crops -> 0.5 (:218-219).
* chunking (:224-238): crops [0:32], [32:64], [64:90] scored by separate
  model calls, so crop j uses pos slot j - chunk_start; crops >= 90 dropped.
"""
from __future__ import annotations

import numpy as np

f32 = np.float32


def sigmoid32(x):
    x = np.asarray(x, f32)
    return (f32(1) / (f32(1) + np.exp(-x))).astype(f32)


def video_score(logits) -> float:
    logits = np.asarray(logits, f32).reshape(-1, 2)
    n = logits.shape[0]
    if n <= 2:
        return 0.5
    p = sigmoid32(logits)
    f = f32(0)
    r = f32(0)
    for i in range(n):
        f = f32(f + p[i, 0])
        r = f32(r + p[i, 1])
    f, r = f32(f / f32(n)), f32(r / f32(n))
    return float(f if f > r else abs(f32(1) - r))


def chunk_slots(n: int) -> np.ndarray:
    n = min(n, 90)
    return np.array([j if j < 32 else (j - 32 if j < 64 else j - 64) for j in range(n)], np.int32)
