"""Drop-in for ``CViT-main/model/cvit.py``.

The reference imports its model with ``sys.path.insert(1, 'model'); from cvit
import CViT`` (cvit_prediction.py:20,24; cvit_train.py:15,19).  Pointing that
path at this directory swaps in the gfx950 HIP implementation with the same
constructor, state_dict and forward contract.
"""
import os
import sys

_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if _ROOT not in sys.path:
    sys.path.insert(0, _ROOT)

from fac_fake_amd.cvit import CViT  # noqa: E402,F401

__all__ = ["CViT"]
