"""Host side of the per-video prediction (CViT-main/cvit_prediction.py:153-281).

The reference runs, per video: face crops (uint8 RGB [N<=29,224,224,3]) ->
``.float()`` -> NCHW -> per-image ``Normalize(x/255)`` -> ``model`` on the
chunks [0:32], [32:64], [64:90] under ``no_grad`` -> ``pred_sig`` ->
``pre_process_prediction`` -> ``.item()``.

Here the crops go to the GPU once as uint8 (4x fewer bytes than the
reference's fp32 H2D copy at :209) and one ``forward_u8`` call covers every
chunk: chunk slots are passed as ``pos_index`` (slot = index within its
chunk, which is what three separate ``model(chunk)`` calls give each crop).
The four helper functions keep the reference's names and semantics.
"""
from __future__ import annotations

import numpy as np
import torch

CHUNKS = ((0, 32), (32, 64), (64, 90))   # cvit_prediction.py:226-238
MAX_CROPS = 90                          # crops past index 90 are never scored (:236)
EMPTY_SCORE = 0.5                       # no face found (:218-219) / <=2 crops (:280-281)


def non_empty(dfdc_tensor, df_len, lower_bound, upper_bound, flag):
    """Slice [lower_bound, min(df_len, upper_bound)) when flag, else everything (:245-255)."""
    if flag is True:
        return dfdc_tensor[lower_bound:min(df_len, upper_bound)]
    if flag is False:
        return dfdc_tensor
    return []


def pred_sig(dfdc_tensor: torch.Tensor) -> torch.Tensor:
    """Per-logit sigmoid of the squeezed logits (:258-259) - not a softmax."""
    return torch.sigmoid(dfdc_tensor.squeeze())


def pred_tensor(dfdc_tensor: torch.Tensor, pre_tensor: torch.Tensor) -> torch.Tensor:
    return torch.cat((dfdc_tensor, pre_tensor), 0)


def pre_process_prediction(y_pred: torch.Tensor) -> torch.Tensor:
    """Video score from per-crop probabilities (:266-281).

    More than two rows: f = mean of column 0, r = mean of column 1 (running
    fp32 sums in crop order, as Python's ``sum`` over 0-d tensors does);
    return f if f > r else |1 - r|.  Two rows or fewer (incl. one crop, whose
    squeezed probabilities have length 2): 0.5.
    """
    if len(y_pred) <= 2:
        return torch.tensor(EMPTY_SCORE)
    n = len(y_pred)
    f_sum, r_sum = y_pred[0, 0], y_pred[0, 1]
    for i in range(1, n):
        f_sum = f_sum + y_pred[i, 0]
        r_sum = r_sum + y_pred[i, 1]
    f_c, r_c = f_sum / n, r_sum / n
    return f_c if f_c > r_c else abs(1 - r_c)


def chunk_slots(n: int) -> np.ndarray:
    """pos_embedding slot of crop j when the reference scores n crops in chunks."""
    n = min(n, MAX_CROPS)
    slots = np.empty(n, dtype=np.int32)
    for lo, hi in CHUNKS:
        if lo < n:
            slots[lo:min(n, hi)] = np.arange(min(n, hi) - lo, dtype=np.int32)
    return slots


def dense_slots(n: int, offset: int = 0) -> np.ndarray:
    """Slots for dense mode (every crop scored): global index mod 32."""
    return ((np.arange(n, dtype=np.int64) + offset) % 32).astype(np.int32)


def predict_crops(model, crops: torch.Tensor) -> float:
    """Score one video's face crops like ``predict`` (:202-242) does after detection.

    ``crops``: uint8 [N,224,224,3] RGB (host or device).  Returns the video
    probability as a Python float; < 0.5 means REAL, >= 0.5 FAKE (:289-292).
    """
    n = int(crops.shape[0])
    if n == 0:
        return float(EMPTY_SCORE)
    n = min(n, MAX_CROPS)
    dev = torch.device("cuda", torch.cuda.current_device()) if not crops.is_cuda else crops.device
    x = crops[:n].to(dev, non_blocking=True)
    slots = torch.from_numpy(chunk_slots(n))
    with torch.no_grad():
        logits = model.forward_u8(x, pos_index=slots)
    return float(pre_process_prediction(pred_sig(logits.float().cpu())))


def label(score: float) -> str:
    return "REAL" if score < 0.5 else "FAKE"
