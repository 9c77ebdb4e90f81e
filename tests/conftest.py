import os
import sys
import tempfile

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

# Keep MIOpen's solver choices (its per-user find-db) private to this test session, so
# convolutions run under cudnn.deterministic here do not steer later processes (bench.py).
os.environ.setdefault("MIOPEN_USER_DB_PATH", tempfile.mkdtemp(prefix="ssq_test_miopen_"))

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); run with -m gpu")


def load_golden(name):
    return dict(np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False))


@pytest.fixture(scope="session")
def golden():
    return load_golden


def assert_walk_bounded(dev, tight, budget, frac=0.005, what=""):
    """Learned parameters follow the reference trajectory to `tight`, except entries whose
    gradient nearly cancels: Adam turns the sign of that residue into +-lr steps, in the
    reference on its CPU as here, and which entries do so depends on the fp32 summation
    order of the box's conv solvers.  At most max(1, frac * size) such entries, none
    beyond Adam's step budget.  Returns how many walked."""
    dev = np.asarray(dev, dtype=np.float64)
    n_off = int((dev > tight).sum())
    assert n_off <= max(1, round(frac * dev.size)), (what, n_off, float(dev.max(initial=0.0)))
    assert float(dev.max(initial=0.0)) <= budget, (what, float(dev.max(initial=0.0)))
    return n_off
