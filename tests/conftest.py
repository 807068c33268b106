import json
import sys
from pathlib import Path

import numpy as np
import pytest

REPO = Path(__file__).resolve().parent.parent
PKG = REPO / "reliable-udp_amd"
GOLDEN = REPO / "tests" / "golden"
for p in (str(REPO), str(PKG)):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a HIP device (MI355X) and librudp.so")
    config.addinivalue_line("markers", "slow: full-size (BASELINE config) checks")


@pytest.fixture(scope="session")
def golden_small():
    with np.load(GOLDEN / "frames_small.npz") as z:
        return {k: z[k] for k in z.files}


@pytest.fixture(scope="session")
def edge_cases():
    return json.loads((GOLDEN / "edge_cases.json").read_text())


@pytest.fixture(scope="session")
def digests():
    path = GOLDEN / "digests.json"
    if not path.exists():
        pytest.skip("digests.json not generated")
    return json.loads(path.read_text())


@pytest.fixture(scope="session")
def wire_trace():
    return json.loads((GOLDEN / "wire_trace.json").read_text())


def small_lengths(golden):
    return sorted({int(k.split("_")[0][1:]) for k in golden if k.endswith("_frames5")})


@pytest.fixture(scope="session")
def cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    return torch.device("cuda", 0)


@pytest.fixture(scope="session")
def golden_varlen():
    with np.load(GOLDEN / "varlen.npz") as z:
        return {k: z[k] for k in z.files}


def split_by_lengths(buf, lengths):
    off = np.concatenate([[0], np.cumsum(lengths)]).astype(np.int64)
    return [bytes(buf[off[i]:off[i + 1]]) for i in range(len(lengths))], off


@pytest.fixture(scope="session")
def golden_dedup():
    with np.load(GOLDEN / "dedup.npz") as z:
        return {k: z[k] for k in z.files}


@pytest.fixture(autouse=True)
def _product_library_after_each_test():
    """Tests of the non-default kernel forms switch the batch API to the
    diagnostics build (rudp._native.tools_lib()); every test ends on librudp.so."""
    yield
    from rudp import _native
    _native.use_product()
