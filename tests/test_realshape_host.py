"""CPU side of the real-shape parity cases (no GPU): the seeded nets rebuilt from
tests/golden/realshape.py have the reference's module layout, and the BN-folded weights
our QuantModel produces are hash-identical to the reference's (real_<case>.npz)."""
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden"))
import realshape as RS  # noqa: E402
from test_realshape_gpu import named_qms, real_qnn  # noqa: E402


@pytest.mark.parametrize("case", list(RS.CASES))
def test_real_seeded_fold_matches_reference(golden, case):
    from shiftedscalequantization_amd import quant as Q
    g = golden(f"real_{case}")
    qnn = real_qnn(Q, case, g, cuda=False)
    qms = named_qms(qnn.model[0], Q)
    assert [n for n, _ in qms] == [str(s) for s in g["qms"]]
    for n, m in qms:
        assert RS.sha(m.org_weight.detach().numpy()) == str(g[f"{n}_w_sha"][0]), n
        assert RS.sha(m.org_bias.detach().numpy()) == str(g[f"{n}_b_sha"][0]), n


def test_realshape_rng_is_integer_exact():
    """xnormal / xuniform are integer draws + exactly rounded float32 ops: a fixed seed
    gives fixed bits (pinned values), whatever the CPU."""
    import torch
    g = torch.Generator().manual_seed(1)
    a = RS.xnormal(g, (4,)).numpy()
    g = torch.Generator().manual_seed(1)
    b = RS.xnormal(g, (4,)).numpy()
    assert np.array_equal(a, b)
    x = RS.calib_input("r50_layer1_0")
    assert x.shape == (RS.N_CALI, 64, 6, 6) and float(x.min()) == 0.0
    assert abs(float(RS.xnormal(torch.Generator().manual_seed(3), (100000,)).std()) - 1.0) < 0.01
