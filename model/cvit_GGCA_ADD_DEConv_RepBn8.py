"""Drop-in for ``CViT-main/model/cvit_GGCA_ADD_DEConv_RepBn8.py``.

With the reference's ``sys.path.insert(1, 'model')`` pointed at this
directory, ``from cvit_GGCA_ADD_DEConv_RepBn8 import CViT`` gives the gfx950
HIP implementation with the same constructor, state_dict and forward contract
(fac_fake_amd/repbn8.py).
"""
import os
import sys

_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if _ROOT not in sys.path:
    sys.path.insert(0, _ROOT)

from fac_fake_amd.repbn8 import CViT  # noqa: E402,F401

__all__ = ["CViT"]
