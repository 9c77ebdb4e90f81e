"""Diagnostic: the BRECQ act phase against recon_brecq_long.npz iteration by iteration.
Runs the weight phase (as the parity test does), then the act phase with every iteration's
loss and act deltas recorded; writes gpurun_out/brecq_act_diag.npz for an offline diff
against the fixture."""
import importlib
import os
import sys

import numpy as np
import torch

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, R)
sys.path.insert(0, os.path.join(R, "tests"))
import test_recon_gpu as T  # noqa: E402
from shiftedscalequantization_amd import quant as Q  # noqa: E402

BR = importlib.import_module("shiftedscalequantization_amd.quant.block_recon")
E = importlib.import_module("shiftedscalequantization_amd.quant._engine")
name = sys.argv[1] if len(sys.argv) > 1 else "recon_brecq_long"
g = np.load(os.path.join(R, "tests", "golden", name + ".npz"))
qnn = T.build_qnn(Q, g)
block = qnn.model[3]
if "conv1_gamma" in g.files:
    for n in ("conv1", "conv2", "downsample"):
        m = getattr(block, n)
        with torch.no_grad():
            m.alpha_out.copy_(T.dev(g[n + "_gamma"]))
            m.beta_out.copy_(T.dev(g[n + "_phi"]))
cali = T.dev(g["cali"])
seen = []
orig_rec = BR.LossFunction.record


def spy(self, rec, rnd, b):
    r = orig_rec(self, rec, rnd, b)
    seen.append(float(r))
    return r


BR.LossFunction.record = spy
torch.manual_seed(1005)
Q.block_reconstruction(qnn, block, cali, batch_size=8, iters=len(g["w_total_loss"]), weight=0.01,
                       asym=True, b_range=(20, 2), warmup=0.2, act_quant=False, opt_mode="mse")
w_seen = list(seen)
qnn.set_quant_state(True, True)
with torch.no_grad():
    qnn(cali[:8])
qnn.disable_network_output_quantization()
aqs = [block.act_quantizer] + [m.act_quantizer for m in (block.conv1, block.conv2, block.downsample)
                               if m.act_quantizer.delta is not None]
deltas, lrs, grads = [], [], []
E.ITER_PROBE[0] = lambda i, ps: (deltas.append([float(q.delta) for q in aqs]),
                                 grads.append([float(p.grad) if p.grad is not None else np.nan for p in ps]))
seen.clear()
torch.manual_seed(1005)
Q.block_reconstruction(qnn, block, cali, batch_size=8, iters=len(g["a_total_loss"]), act_quant=True,
                       opt_mode="mse", lr=4e-4, p=2.4)
E.ITER_PROBE[0] = None
out = os.path.join(R, "gpurun_out", "brecq_act_diag_%s%s.npz" % (name, os.environ.get("DIAG_TAG", "")))
os.makedirs(os.path.dirname(out), exist_ok=True)
np.savez(out, w_seen=np.array(w_seen), a_seen=np.array(seen), deltas=np.array(deltas),
         grads=np.array(grads))
a = np.array(seen)
rel = np.abs(a - g["a_total_loss"]) / np.abs(g["a_total_loss"])
print("act loss rel err: first > 1e-5 at", int(np.argmax(rel > 1e-5)) if np.any(rel > 1e-5) else None,
      "max", rel.max(), "final delta", deltas[-1], "golden", g["a_delta"])
