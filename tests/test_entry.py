"""The video-level entry point (cvit_prediction.py at the repo root, the
drop-in for CViT-main/cvit_prediction.py:73-83,153-242,283-371)."""
import json
import sys
from pathlib import Path

import numpy as np
import pytest
import torch

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))


def test_csv_matches_the_reference_pandas_output(tmp_path):
    """write_predictions == pd.DataFrame({filename, label}).to_csv(index=False) (:341-343)."""
    import pandas as pd
    import cvit_prediction as cp
    names = ["a.mp4", "b,c.mp4", "d.mp4", "e.mp4"]
    preds = [0.5, 0.123456789012345, torch.tensor(0.7300000190734863).item(), 1e-9]
    p = cp.write_predictions(names, preds, tmp_path / "ours.csv")
    pd.DataFrame({"filename": names, "label": preds}).to_csv(tmp_path / "ref.csv", index=False)
    assert p.read_text() == (tmp_path / "ref.csv").read_text()
    assert cp.real_or_fake(names, preds) == ["FAKE", "REAL", "FAKE", "REAL"]
    meta = {"a.mp4": 0, "b,c.mp4": 1, "d.mp4": 1, "e.mp4": 1}
    # score < 0.5 counts as 1 (:360-364): a 0 vs 0, b,c 1 vs 1, d 0 vs 1, e 1 vs 1
    assert cp.prediction_accuracy(p, meta) == 0.75


def test_read_video_face_locations_order(tmp_path):
    """face_recognition's (top, right, bottom, left) maps to the crop box (left, top, right, bottom)."""
    import cvit_prediction as cp
    frames = np.zeros((2, 40, 60, 3), np.uint8)
    np.savez(tmp_path / "v.npz", frames=frames, face_locations=np.array([[1, 5, 30, 25, 10]], np.int32))
    fr, boxes = cp.read_video(tmp_path / "v.npz")
    assert fr.shape == (2, 40, 60, 3) and boxes.tolist() == [[1, 10, 5, 30, 25]]
    np.savez(tmp_path / "w.npz", frames=frames, boxes=np.array([[0, 1, 2, 3, 4]], np.int32))
    assert cp.read_video(tmp_path / "w.npz")[1].tolist() == [[0, 1, 2, 3, 4]]


def test_helpers_loader_constants():
    sys.path.insert(1, str(REPO / "helpers"))
    import loader
    assert loader.mean == [0.485, 0.456, 0.406] and loader.std == [0.229, 0.224, 0.225]


@pytest.mark.gpu
def test_predict_on_video_end_to_end(tmp_path):
    """predict_on_video over a folder of decoded videos: each score is
    predict_video's reference-mode score, the CSV holds them in order, and a
    video without faces scores 0.5 (:218-219)."""
    import cvit_prediction as cp
    from fac_fake_amd.video import predict_video, synthetic_video
    cp.load_model(None, "fp16", "cuda:0")
    names = []
    want = []
    for i, (n, seed) in enumerate(((60, 3), (120, 5), (40, 7))):
        frames, boxes = synthetic_video(n, 360, 640, seed=seed, device="cuda:0")
        if i == 2:
            boxes = boxes[:0]
        name = f"v{i}.npz"
        np.savez(tmp_path / name, frames=frames.cpu().numpy(), boxes=boxes)
        names.append(name)
        want.append(predict_video(cp.model, frames, boxes, mode="reference"))
    cp.sample = str(tmp_path)
    got = cp.predict_on_video(names, num_workers=1)
    assert got == want and got[2] == 0.5
    # several reader threads, and groups smaller than the videos' crop total
    # (one forward per video): the same scores, in order
    assert cp.predict_on_video(names, num_workers=3) == want
    assert cp.predict_on_video(names, num_workers=2, batch=8) == want
    out = cp.write_predictions(names, got, tmp_path / "pred.csv")
    rows = out.read_text().splitlines()
    assert rows[0] == "filename,label" and len(rows) == 4
    assert json.loads("[" + ",".join(r.split(",")[1] for r in rows[1:]) + "]") == got
