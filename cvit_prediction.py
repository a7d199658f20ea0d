"""Video-level entry point: the drop-in for ``CViT-main/cvit_prediction.py``.

The reference script scores every ``.mp4`` of a folder (``predict_on_video``,
cvit_prediction.py:73-83, from ``__main__`` :300-343): per video ``predict``
(:153-242) reads frames with cv2, finds faces with face_recognition, crops /
resizes them (``face_face_rec`` :106-121), runs the CViT on the crops in
chunks of 32 and reduces the per-crop sigmoids to one score
(``pre_process_prediction`` :266-281); the scores go to a ``filename,label``
CSV (:341-343, "label" is the score) and, with a metadata file, an accuracy
(:346-371).

Video decoding (cv2) and face detection (dlib HOG / BlazeFace / MTCNN) are
outside this path (only the crop/resize is in scope),
so a "video file" here is the decoded video plus its face locations: an
``.npz`` holding

* ``frames``: uint8 [F, H, W, 3], BGR as ``cv2.VideoCapture.read`` returns;
* ``face_locations``: int32 [n, 5] = (frame, top, right, bottom, left), what
  ``face_recognition.face_locations(frame)`` returns per frame, or ``boxes``:
  int32 [n, 5] = (frame, left, top, right, bottom).

From there everything runs on the GPU (fac_fake_amd/video.py): the frame
schedule of :165-198, crop + INTER_AREA + channel swap (``fac_crop_resize_u8``),
the CViT forward with the chunk slots of :224-238, and the score.  The names,
arguments and return values of the reference's functions are kept.
"""
from __future__ import annotations

import argparse
import csv
import json
import os
import sys
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path

import numpy as np
import torch

sys.path.insert(0, str(Path(__file__).resolve().parent))

from fac_fake_amd.prediction import (label, non_empty, pre_process_prediction, pred_sig,  # noqa: E402,F401
                                     pred_tensor)
from fac_fake_amd.video import (MAX_CROPS_REFERENCE, crop_faces, predict_video, score_selected,  # noqa: E402
                                select_reference)

mean = [0.485, 0.456, 0.406]    # cvit_prediction.py:41 (fused into conv1 here)
std = [0.229, 0.224, 0.225]     # cvit_prediction.py:42
sample = "."                    # folder of videos (cvit_prediction.py:50)
save_csv_path = "./wprediction/cvit.csv"   # :54
model = None                    # set by load_model() (the reference builds it at import, :62-70)
device = "cuda" if torch.cuda.is_available() else "cpu"


def load_model(weights: str | None = None, dtype: str = "fp16", dev: str | None = None):
    """``CViT(224, 7, 2, 512, 1024, 6, 8, 2048)`` + ``load_state_dict`` + ``eval``
    (cvit_prediction.py:62-70).  ``weights``: a state_dict checkpoint as
    ``cvit_train.py:210`` saves it (loaded with ``weights_only=True``), or
    None for the deterministic synthetic weights (the reference ships no
    trained checkpoint)."""
    global model
    from fac_fake_amd.cvit import CViT
    from fac_fake_amd.weights import make_state_dict
    m = CViT(image_size=224, patch_size=7, num_classes=2, channels=512, dim=1024, depth=6, heads=8, mlp_dim=2048,
             dtype=dtype)
    if weights:
        sd = torch.load(weights, map_location="cpu", weights_only=True)
    else:
        sd = {k: torch.from_numpy(np.asarray(v)) for k, v in make_state_dict(0).items()}
    m.load_state_dict(sd)
    m.to(dev or device)
    m.eval()
    model = m
    return m


def read_video(filename: str):
    """The decoded video container: (frames uint8 [F,H,W,3] BGR, boxes int32
    [n,5] as (frame, left, top, right, bottom))."""
    with np.load(filename, allow_pickle=False) as z:
        frames = z["frames"]
        if "boxes" in z:
            boxes = z["boxes"].astype(np.int32).reshape(-1, 5)
        else:
            fl = z["face_locations"].astype(np.int32).reshape(-1, 5)    # frame, top, right, bottom, left
            boxes = np.stack([fl[:, 0], fl[:, 4], fl[:, 1], fl[:, 2], fl[:, 3]], 1).astype(np.int32)
    if frames.dtype != np.uint8 or frames.ndim != 4 or frames.shape[3] != 3:
        raise ValueError(f"{filename}: frames must be uint8 [F,H,W,3], got {frames.dtype} {frames.shape}")
    return frames, boxes


def face_face_rec(frame, face_locations):
    """Crops of one frame (cvit_prediction.py:106-121): the first 5 face
    locations (top, right, bottom, left), ``frame[top:bottom, left:right]``
    -> INTER_AREA 224x224 -> channel swap, as uint8 [n,224,224,3] (on the
    GPU), or ``([], 0)`` when there is no face."""
    locs = list(face_locations)[:5]
    if not locs:
        return [], 0
    fr = torch.as_tensor(np.ascontiguousarray(frame)).to(device).unsqueeze(0)
    boxes = np.array([[0, l, t, r, b] for (t, r, b, l) in locs], np.int32)
    return crop_faces(fr, boxes), len(locs)


def predict(filename, mtcnn=None, mode: str = "reference"):
    """Score of one video, a float (< 0.5 REAL, >= 0.5 FAKE), as
    cvit_prediction.py:153-242 returns it; 0.5 when no face is found.
    ``mtcnn`` is accepted for signature compatibility and unused, as in the
    reference's live path (:180-187 is commented out)."""
    if model is None:
        raise RuntimeError("call load_model() first (the reference builds its model at import)")
    frames, boxes = read_video(filename)
    # host frames: predict_video uploads only the frames its crops come from
    return predict_video(model, frames, boxes, mode=mode)


def predict_on_video(dfdc_filenames, num_workers, batch: int = 256):
    """Scores of the videos ``sample/<filename>`` in order (:73-83).

    The reference maps ``predict`` over a ``ThreadPoolExecutor(num_workers)``
    (one worker, :303), i.e. one <= 29-crop forward per video.  Here the
    ``num_workers`` threads only read the files and keep each video's crop
    selection and the frames it needs (``select_reference``); the GPU work
    stays on the calling thread, which scores the crops of consecutive videos
    together in forwards of up to ``batch`` crops (``score_selected``: each
    video keeps its own slots 0..n-1, one segmented score launch per group).
    Every score is bit-identical to ``predict`` on that video alone."""
    if model is None:
        raise RuntimeError("call load_model() first (the reference builds its model at import)")

    def load(i):
        frames, boxes = read_video(os.path.join(sample, dfdc_filenames[i]))
        return select_reference(frames, boxes)

    # read-ahead is bounded: at most num_workers + 1 loaded videos wait for
    # the GPU (each holds its selected host frames, ~190 MB at 1080p; the
    # reference's threads only ever hold float scores)
    from collections import deque
    workers = max(1, int(num_workers))
    n = len(dfdc_filenames)

    def items(ex):
        pending, nxt = deque(), 0
        while nxt < n or pending:
            while nxt < n and len(pending) < workers + 1:
                pending.append(ex.submit(load, nxt))
                nxt += 1
            yield pending.popleft().result()

    predictions, group, ncrops = [], [], 0
    with ThreadPoolExecutor(max_workers=workers) as ex:
        for item in items(ex):
            if group and ncrops + len(item[1]) > batch:
                predictions += score_selected(model, group, batch)
                group, ncrops = [], 0
            group.append(item)
            ncrops += len(item[1])
        if group:
            predictions += score_selected(model, group, batch)
    return predictions


def real_or_fake(filenames, predictions):
    """Per-video labels, REAL if the score < 0.5 else FAKE (:289-296)."""
    return [label(float(p)) for p in predictions]


def write_predictions(filenames, predictions, path=None):
    """``pd.DataFrame({"filename": ..., "label": ...}).to_csv(path, index=False)``
    (:341-343): a header line, then ``filename,score`` rows, floats in
    Python's shortest round-trip form as pandas writes them."""
    path = Path(path or save_csv_path)
    path.parent.mkdir(parents=True, exist_ok=True)
    with open(path, "w", newline="") as f:
        w = csv.writer(f, lineterminator="\n")
        w.writerow(["filename", "label"])
        for fn, p in zip(filenames, predictions):
            w.writerow([fn, repr(float(p))])
    return path


def prediction_accuracy(csv_path, metadata) -> float:
    """:346-371: a score < 0.5 counts as 1, else 0, compared with
    ``metadata[filename]``; returns the fraction correct."""
    data = json.loads(Path(metadata).read_text()) if isinstance(metadata, (str, Path)) else metadata
    rows = list(csv.DictReader(open(csv_path)))
    score = 0
    for r in rows:
        pred = 1 if float(r["label"]) < 0.5 else 0
        if pred == data[r["filename"]]:
            score += 1
    return score / len(rows) if rows else 0.0


def main(argv=None):
    global sample, save_csv_path
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--sample", default=sample, help="folder of decoded videos (.npz)")
    ap.add_argument("--csv", default=save_csv_path)
    ap.add_argument("--weights", default=None, help="CViT state_dict checkpoint (default: synthetic weights)")
    ap.add_argument("--dtype", default="fp16", choices=["fp16", "bf16"])
    ap.add_argument("--metadata", default=None, help="json {filename: 0/1} for the accuracy")
    ap.add_argument("--num-workers", type=int, default=1)
    args = ap.parse_args(argv)
    sample, save_csv_path = args.sample, args.csv
    load_model(args.weights, args.dtype)
    filenames = sorted(x for x in os.listdir(sample) if x.endswith(".npz"))
    predictions = predict_on_video(filenames, num_workers=args.num_workers)
    print(predictions)
    for fn, lb in zip(filenames, real_or_fake(filenames, predictions)):
        print("Filname:", fn, lb)
    write_predictions(filenames, predictions, save_csv_path)
    if args.metadata:
        print(f"prediction Acc:  {prediction_accuracy(save_csv_path, args.metadata) * 100}%")
    return predictions


__all__ = ["MAX_CROPS_REFERENCE", "face_face_rec", "load_model", "non_empty", "pre_process_prediction", "pred_sig",
           "pred_tensor", "predict", "predict_on_video", "prediction_accuracy", "read_video", "real_or_fake",
           "write_predictions"]

if __name__ == "__main__":
    main()
