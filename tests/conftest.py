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
