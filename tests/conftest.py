import json
import os
import sys
from pathlib import Path

import numpy as np
import pytest

REPO = Path(__file__).resolve().parents[1]
GOLDEN = REPO / "tests" / "golden"
sys.path.insert(0, str(REPO))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU and the built HIP library")


def pytest_collection_modifyitems(config, items):
    # keep GPU tests in this one process (the box allows few GPU processes)
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(pytest.mark.timeout(900))


@pytest.fixture(scope="session")
def sd():
    from fac_fake_amd.weights import make_state_dict
    return make_state_dict(0)


@pytest.fixture(scope="session")
def golden():
    def _load(name):
        p = GOLDEN / name
        if p.suffix == ".json":
            return json.loads(p.read_text())
        return dict(np.load(p, allow_pickle=False))
    return _load


ENVELOPE_MARGIN = 1.25
# The HIP path is not the emulation: fp32 summation order flips a 16-bit
# rounding by one ulp on a few % of the activations (the per-kernel tests
# bound it), which moves a probability by up to 2.5e-4 beyond the emulated
# envelope on the few-output fixtures (measured: S3D 20x224 bf16, 5.8e-4 vs
# an emulated 3.3e-4).  2x that is added to the bf16 gates.
ORDER_NOISE = 5e-4


def bf16_gate(envelope: float) -> float:
    return ENVELOPE_MARGIN * envelope + ORDER_NOISE


@pytest.fixture(scope="session")
def tol16():
    """End-to-end probability tolerance of a golden fixture: fp16 at the
    north-star bar (1e-3); bf16 at 1.25x the oracle's emulated bf16 rounding
    envelope on that fixture's own inputs (tests/golden/bf16_envelope.json,
    tools/bf16_envelope.py) plus ORDER_NOISE, so a bf16-only regression
    cannot hide in a flat 1e-2."""
    env = json.loads((GOLDEN / "bf16_envelope.json").read_text())

    def _tol(dt, fixture):
        if dt == "fp16":
            return 1e-3
        return bf16_gate(env["bf16"][fixture])
    return _tol


@pytest.fixture(scope="session", autouse=True)
def built_lib():
    """(Re)build libfac_cvit.so when any source is newer than it (mtime-checked,
    hipcc cross-compiles without a GPU), so a stale shipped .so is never what
    gets tested.  On a box without hipcc the shipped library is used as is."""
    from fac_fake_amd import build
    try:
        build.build()
    except RuntimeError as e:
        if not build.LIB.exists() or "hipcc not found" not in str(e):
            raise
    return build.LIB


@pytest.fixture(scope="session")
def torch_threads():
    import torch
    torch.set_num_threads(min(16, os.cpu_count() or 8))
    return torch
