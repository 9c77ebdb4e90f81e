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
