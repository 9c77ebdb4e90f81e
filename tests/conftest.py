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


def assert_hard_flips_bounded(what, what_ref, v, v_ref, budget, what_name=""):
    """AdaRound's hard weights against the reference's: a code may differ only where the
    rounding decision (V >= 0) flipped, a decision may flip only where the reference's V is
    within Adam's walk budget of zero (its gradient nearly cancels, so either side is the
    fp32 summation order's call), and with no flip the hard weights are bit-identical.
    Returns the number of flipped decisions."""
    what, what_ref = np.asarray(what, np.float32), np.asarray(what_ref, np.float32)
    v = np.asarray(v, np.float32).reshape(what.shape)
    v_ref = np.asarray(v_ref, np.float32).reshape(what.shape)
    flip = (v >= 0) != (v_ref >= 0)
    assert np.all(np.abs(v_ref[flip]) <= budget), (what_name, v_ref[flip])
    differs = what.view(np.int32) != what_ref.view(np.int32)
    assert not np.any(differs & ~flip), (what_name, int((differs & ~flip).sum()))
    if not flip.any():
        assert not differs.any(), what_name
    return int(flip.sum())


def assert_shift_flips_bounded(what, what_ref, alpha, alpha_ref, budget, what_name=""):
    """adaShift's hard weights (the argmax shift of each alpha row, channelQuant.py:99-106)
    against the reference's: a code may differ only in an alpha row (conv: input channel;
    fc: element) whose argmax flipped, a row may flip only where the reference's top-two
    logit margin is within twice Adam's walk budget, and with no flip the hard weights are
    bit-identical.  Returns the number of flipped rows."""
    what, what_ref = np.asarray(what, np.float32), np.asarray(what_ref, np.float32)
    alpha, alpha_ref = np.asarray(alpha, np.float32), np.asarray(alpha_ref, np.float32)
    flip = alpha.argmax(-1) != alpha_ref.argmax(-1)
    top2 = np.sort(alpha_ref, axis=-1)[..., -2:]
    margin = top2[..., 1] - top2[..., 0]
    assert np.all(margin[flip] <= 2 * budget), (what_name, margin[flip])
    differs = what.view(np.int32) != what_ref.view(np.int32)
    if alpha.ndim == 2:                       # conv: alpha (Ci, S), weight (Co, Ci, ...)
        differs_rows = differs.reshape(what.shape[0], what.shape[1], -1).any(axis=(0, 2))
    else:                                     # fc: alpha (Co, Ci, S), weight (Co, Ci)
        differs_rows = differs.reshape(alpha.shape[:-1])
    assert not np.any(differs_rows & ~flip), (what_name, int((differs_rows & ~flip).sum()))
    if not flip.any():
        assert not differs.any(), what_name
    return int(flip.sum())
