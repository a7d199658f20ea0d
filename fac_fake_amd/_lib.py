"""ctypes binding of libfac_cvit.so (include/fac_cvit.h).

The library is loaded after ``import torch`` so its ``DT_NEEDED
libamdhip64.so.7`` resolves to the HIP runtime torch has already mapped: one
runtime, so torch tensors' device pointers and ``torch.cuda`` streams can be
handed to the C ABI as plain integers.  There is no CPU fallback: if the
library is missing or cannot load, every entry point raises.
"""
from __future__ import annotations

import ctypes
import os
from pathlib import Path

import torch  # noqa: F401  (must precede the dlopen below, see module doc)

LIB_PATH = Path(os.environ.get("FAC_CVIT_LIB", Path(__file__).resolve().parent / "libfac_cvit.so"))

FAC_OK = 0
STATUS = {0: "FAC_OK", -1: "FAC_ERR_ARG", -2: "FAC_ERR_SHAPE", -3: "FAC_ERR_MISSING", -4: "FAC_ERR_HIP",
          -5: "FAC_ERR_NOT_LOADED", -6: "FAC_ERR_OOM"}
DTYPES = {"bf16": 0, "fp16": 1}

# Every symbol include/fac_cvit.h declares, with its ctypes signature.
SIGNATURES = {
    "fac_create": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_void_p)]),
    "fac_load_weights": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]),
    "fac_reserve": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]),
    "fac_workspace_bytes": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(ctypes.c_size_t)]),
    "fac_forward_nchw_f32": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p,
                                            ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    "fac_forward_nhwc_u8": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p,
                                           ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    "fac_forward_nhwc_u8_pipelined": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int,
                                                     ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                                     ctypes.c_void_p, ctypes.c_void_p]),
    "fac_pipeline_join": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]),
    "fac_debug_features_u8": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                                             ctypes.c_void_p, ctypes.c_void_p]),
    "fac_debug_conv": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p,
                                      ctypes.c_void_p]),
    "fac_debug_tail": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p,
                                      ctypes.c_void_p, ctypes.c_void_p]),
    "fac_debug_gemm": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                                      ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                      ctypes.c_int, ctypes.c_int, ctypes.c_void_p]),
    "fac_profile_forward_u8": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p,
                                              ctypes.c_void_p, ctypes.POINTER(ctypes.c_float), ctypes.c_int,
                                              ctypes.c_void_p]),
    "fac_stem_event_ms": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_float),
                                         ctypes.POINTER(ctypes.c_int)]),
    "fac_check_device_errors": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_int)]),
    "fac_video_score": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]),
    "fac_video_score_seg": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p,
                                           ctypes.c_void_p]),
    "fac_crop_resize_u8": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                                          ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]),
    "fac_forward_features": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p,
                                            ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    # include/fac_ops.h
    "fac_conv_nd": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p]),
    "fac_conv_s2d4_clip": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                          ctypes.c_void_p]),
    "fac_conv_s2d4_clip_u8": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                                             ctypes.c_int, ctypes.c_void_p]),
    "fac_s3d_base0_u8": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                                        ctypes.c_int, ctypes.c_void_p]),
    "fac_conv_nd_dual": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    "fac_sep_tiny": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    "fac_sep_mid": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    "fac_bottleneck_pw2": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    "fac_conv_weight_layout": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                              ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int)]),
    "fac_pool_nd": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p]),
    "fac_pack_input": (ctypes.c_int, [ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                      ctypes.c_float, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int,
                                      ctypes.c_void_p]),
    "fac_pack_input_s2d": (ctypes.c_int, [ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                          ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_float,
                                          ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    "fac_kan_linear": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                                      ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                      ctypes.c_void_p]),
    "fac_kan_scratch_bytes": (ctypes.c_size_t, [ctypes.c_int, ctypes.c_int, ctypes.c_int]),
    "fac_sigmoid": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]),
    "fac_conv_nd_split": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                                          ctypes.c_int, ctypes.c_int, ctypes.c_void_p]),
    "fac_conv3x3_packed_elems": (ctypes.c_size_t, [ctypes.c_int, ctypes.c_int, ctypes.c_int]),
    "fac_conv3x3_pack": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                                        ctypes.c_void_p]),
    "fac_conv3x3": (ctypes.c_int, [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                   ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                   ctypes.c_void_p, ctypes.c_void_p]),
    "fac_stem224_pack_conv1": (ctypes.c_int, [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]),
    "fac_stem224": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                   ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                   ctypes.c_int, ctypes.c_void_p]),
    "fac_ggca": (ctypes.c_int, [ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    "fac_set_stem_chunk": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]),
    "fac_set_option": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_int]),
    "fac_last_error": (ctypes.c_char_p, [ctypes.c_void_p]),
    "fac_destroy": (None, [ctypes.c_void_p]),
    "fac_version": (ctypes.c_char_p, []),
}


class TensorDesc(ctypes.Structure):
    _fields_ = [("name", ctypes.c_char_p), ("data", ctypes.c_void_p), ("ndim", ctypes.c_int),
                ("shape", ctypes.c_int64 * 4)]


_lib = None


def load() -> ctypes.CDLL:
    """dlopen libfac_cvit.so once; raise if it is missing (no fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    if not LIB_PATH.exists():
        raise RuntimeError(f"{LIB_PATH} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'`"
                           " (the CViT path has no CPU fallback)")
    lib = ctypes.CDLL(str(LIB_PATH), mode=ctypes.RTLD_GLOBAL)
    overridden = "FAC_CVIT_LIB" in os.environ  # an older build for an A/B run may lack newer entry points
    for name, (res, args) in SIGNATURES.items():
        try:
            fn = getattr(lib, name)
        except AttributeError:
            if not overridden:
                raise

            def _missing(*_a, _n=name):
                raise RuntimeError(f"{LIB_PATH} does not export {_n}")
            setattr(lib, name, _missing)
            continue
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def exports(name: str) -> bool:
    """Whether the loaded library has entry point `name` (only an older build
    selected with FAC_CVIT_LIB for an A/B run can lack one)."""
    return isinstance(getattr(load(), name), ctypes._CFuncPtr)


class FacError(RuntimeError):
    pass


def check(rc: int, ctx=None, what: str = "") -> None:
    if rc != FAC_OK:
        msg = ""
        if ctx:
            m = load().fac_last_error(ctx)
            msg = m.decode() if m else ""
        raise FacError(f"{what} failed: {STATUS.get(rc, rc)} {msg}".strip())
