"""Repeat the prepared adaShift forward / alpha backward of the recon_fused block's three
convs (one multi-segment launch each) with cache-evicting copies in between and report any
run-to-run difference."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
from shiftedscalequantization_amd import kernels as K  # noqa: E402

SHIFTS = [31 / 32, 33 / 32, 1.0]
shapes = [(32, 16, 3, 3), (32, 32, 3, 3), (32, 16, 1, 1)]
if len(sys.argv) > 1:
    shapes = [(64, 64, 3, 3), (64, 64, 3, 3)]
torch.manual_seed(0)
big_a = torch.empty(256 << 20, device="cuda")
big_b = torch.empty_like(big_a)
alphas, entries, gys = [], [], []
for shape in shapes:
    w = torch.randn(shape, device="cuda") * 0.05
    d, z, _ = K.scale_init(w, 2, False, True, "max")
    alpha, beta, _ = K.shift_init(w, d, SHIFTS)
    alpha = alpha + torch.randn_like(alpha) * 0.5
    alphas.append(alpha)
    entries.append((K.AdaShiftPrep(w, beta, d, SHIFTS, 0), d, z, 2, False))
    gys.append(torch.randn_like(w))
regp = torch.tensor([0.1, 5.0], device="cuda")
bad_f = bad_b = 0
for trial in range(30):
    res = []
    for rep in range(3):
        if rep:
            big_b.copy_(big_a)
        am = [a.clone().requires_grad_(True) for a in alphas]
        vals = [torch.zeros(a.shape[0], device="cuda") for a in alphas]
        ys = K.adashift_prepared_multi(am, entries, False, reg=(0.0, 0.0, vals, regp))
        if rep == 2:
            big_b.copy_(big_a)
        torch.autograd.backward(list(ys), gys)
        res.append(([y.detach().clone() for y in ys], [a.grad.clone() for a in am]))
    for rep in (1, 2):
        for k in range(len(shapes)):
            if not torch.equal(res[rep][0][k], res[0][0][k]):
                bad_f += 1
                print("fwd differs", trial, rep, shapes[k], (res[rep][0][k] != res[0][0][k]).sum().item())
            if not torch.equal(res[rep][1][k], res[0][1][k]):
                bad_b += 1
                diff = (res[rep][1][k] != res[0][1][k])
                print("bwd differs", trial, rep, shapes[k], diff.sum().item(),
                      diff.nonzero()[:4].tolist())
    gys = [torch.randn_like(g) for g in gys]
print("fwd mismatches", bad_f, "bwd mismatches", bad_b)
