"""K5p / K6p launch durations of whole ResNet-18 blocks with cold caches, as in the recon
loop (every small kernel there follows an activation-sized pass): each forward + backward of
a block's adaShift is preceded by a 1 GB copy that evicts L2 / MALL.  Run under
rocprofv3 --kernel-trace and summarise with tools/trace_avg.py.
    SSQ_ALPHA_ONE_LAUNCH=0|1 python tools/alpha_cold.py [reps]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from shiftedscalequantization_amd import kernels as K  # noqa: E402
from tools.adashift_bench import BLOCKS, SHIFTS  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 50
    torch.manual_seed(0)
    big_a = torch.empty(256 << 20, device="cuda")
    big_b = torch.empty_like(big_a)
    for name, shapes in BLOCKS.items():
        alphas, entries, gys, vals = [], [], [], []
        for shape in shapes:
            w = torch.randn(shape, device="cuda") * 0.05
            d, z, _ = K.scale_init(w, 2, False, True, "max")
            alpha, beta, _ = K.shift_init(w, d, SHIFTS)
            alphas.append(alpha.requires_grad_(True))
            entries.append((K.AdaShiftPrep(w, beta, d, SHIFTS, 0), d, z, 2, False))
            gys.append(torch.randn_like(w))
            vals.append(torch.zeros(alpha.shape[0], device="cuda"))
        regp = torch.tensor([0.1, 5.0], device="cuda")
        reg = (0.0, 0.0, vals, regp)
        for _ in range(reps):
            big_b.copy_(big_a)
            for a in alphas:
                a.grad = None
            ys = K.adashift_prepared_multi(alphas, entries, False, reg=reg)
            big_b.copy_(big_a)
            torch.autograd.backward(list(ys), gys)
        torch.cuda.synchronize()
        print(name, "done", flush=True)


if __name__ == "__main__":
    main()
