"""fac_fake_amd: MI355X-native (gfx950) CViT per-frame face-forgery inference path.

Drop-in for CViT-main/model/cvit.py + the scoring half of
CViT-main/cvit_prediction.py, with the forward as hand-written HIP/MFMA
kernels behind a C ABI (include/fac_cvit.h, libfac_cvit.so).
"""
from .weights import make_crops, make_state_dict  # noqa: F401

__all__ = ["CViT", "make_state_dict", "make_crops"]


def __getattr__(name):
    if name == "CViT":  # lazy: importing torch + dlopen only when the model is used
        from .cvit import CViT
        return CViT
    raise AttributeError(name)
