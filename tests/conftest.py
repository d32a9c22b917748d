import sys
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parent.parent
GOLDEN = ROOT / "tests" / "golden"
if str(ROOT) not in sys.path:
    sys.path.insert(0, str(ROOT))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run with -m gpu on the GPU box)")


@pytest.fixture(scope="session")
def oracle():
    from oracle.oracle_lib import Oracle
    return Oracle()


@pytest.fixture(scope="session")
def raw_golden():
    with np.load(GOLDEN / "raw_vectors.npz") as z:
        return {k: z[k] for k in z.files}


@pytest.fixture(scope="session")
def tcp4_golden():
    with np.load(GOLDEN / "tcp4_vectors.npz") as z:
        return {k: z[k] for k in z.files}
