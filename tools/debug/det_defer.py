"""Run the fused loop of test_deferred_finalize_bit_identical several times per deferral
mode and print each run's per-iteration losses and final alpha checksums."""
import importlib
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
import test_recon_gpu as T  # noqa: E402
from shiftedscalequantization_amd import quant as Q  # noqa: E402

LRF = importlib.import_module("shiftedscalequantization_amd.quant.layer_recon_fused_shiftedScale")
gpath = os.path.join(os.path.dirname(__file__), "..", "..", "tests", "golden", "recon_fused.npz")
g = np.load(gpath)


from shiftedscalequantization_amd.quant import _engine as E  # noqa: E402


def run(defer, bias_cal=True, trace=None):
    qnn = T.build_qnn(Q, {})
    block = qnn.model[3]
    T.load_block(Q, g, block)
    block.cached_inp_features = [T.dev(g["cached_inp"])]
    block.cached_out_features = [T.dev(g["cached_out"])]
    seen = []
    orig = LRF.FusedScaleLossFunction.bookkeep

    def bk(self, rec):
        seen.append(float(rec.item()))
        return orig(self, rec)
    LRF.FusedScaleLossFunction.bookkeep, prev = bk, LRF.DEFER_FINALIZE
    LRF.DEFER_FINALIZE = defer
    if trace is not None:
        E.ITER_PROBE[0] = lambda i, ps: trace.append(
            (i, [None if q.grad is None else q.grad.detach().clone() for q in ps],
             [q.detach().clone() for q in ps]))
    try:
        torch.manual_seed(1005)
        LRF.block_recon_fused_shiftedScale(block, 12, (0.01, 0.1), qnn, None, verbose=False,
                                           graph=False, bias_cal=bias_cal)
    finally:
        LRF.FusedScaleLossFunction.bookkeep, LRF.DEFER_FINALIZE = orig, prev
        E.ITER_PROBE[0] = None
    al = [getattr(block, n).weight_quantizer.alpha.detach().double().sum().item()
          for n in ("conv1", "conv2", "downsample")]
    ga = [getattr(block, n).alpha_out.detach().double().sum().item() for n in ("conv1", "conv2", "downsample")]
    return np.array(seen), al, ga


import sys as _s
if "--det" in _s.argv:
    torch.backends.cudnn.deterministic = True
tr = [[], []]
for k in range(2):
    run(False, False, tr[k])
for (i, g0, p0), (_, g1, p1) in zip(*tr):
    for j, (a, b) in enumerate(zip(g0, g1)):
        if a is not None and not torch.equal(a, b):
            d = (a != b)
            print(f"iter {i} param {j} shape {tuple(a.shape)} grad differs at {d.sum().item()} entries,"
                  f" first {d.nonzero()[:3].tolist()} vals {a[d][:3].tolist()} vs {b[d][:3].tolist()}")
    for j, (a, b) in enumerate(zip(p0, p1)):
        if not torch.equal(a, b):
            print(f"iter {i} param {j} value differs at {(a != b).sum().item()}")
print("done")
