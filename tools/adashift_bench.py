"""Standalone timing of the adaShift kernels (K5/K6, recomputing vs prepared) on the
ResNet-18 conv shapes: HIP-event average over back-to-back launches on the launch
stream; achieved = 12 B/elem / time.  Prints one JSON line per shape."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from shiftedscalequantization_amd import kernels as K  # noqa: E402

SHIFTS = [31 / 32, 33 / 32, 1.0]
SHAPES = [(64, 64, 3, 3), (128, 128, 3, 3), (256, 256, 3, 3), (512, 512, 3, 3), (512, 256, 3, 3),
          (512, 256, 1, 1)]


def t_ms(fn, reps=20, rounds=5):
    """Device time per call: `reps` calls captured in one HIP graph (no host launch cost),
    replayed `rounds` times; median of the per-replay averages."""
    fn()
    torch.cuda.synchronize()
    graph, ws = torch.cuda.CUDAGraph(), {}
    with K.A.workspace_scope(ws):
        with torch.cuda.graph(graph):
            for _ in range(reps):
                fn()
    graph.replay()
    torch.cuda.synchronize()
    times = []
    for _ in range(rounds):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        graph.replay()
        b.record()
        torch.cuda.synchronize()
        times.append(a.elapsed_time(b) / reps)
    return sorted(times)[len(times) // 2]


BLOCKS = {"layer1.0": [(64, 64, 3, 3)] * 2,
          "layer2.0": [(128, 64, 3, 3), (128, 128, 3, 3), (128, 64, 1, 1)],
          "layer3.0": [(256, 128, 3, 3), (256, 256, 3, 3), (256, 128, 1, 1)],
          "layer4.0": [(512, 256, 3, 3), (512, 512, 3, 3), (512, 256, 1, 1)],
          "layer4.1": [(512, 512, 3, 3)] * 2}


def blocks():
    """The multi-segment launches of a whole ResNet-18 block (the fused loop's form)."""
    torch.manual_seed(0)
    out = {"wgs": os.environ.get("SSQ_PREP_WGS", "1536"), "rows": os.environ.get("SSQ_PREP_ROWS", "8")}
    for name, shapes in BLOCKS.items():
        alphas, entries, gys, vals = [], [], [], []
        n = 0
        for shape in shapes:
            w = torch.randn(shape, device="cuda") * 0.05
            d, z, _ = K.scale_init(w, 2, False, True, "max")
            alpha, beta, _ = K.shift_init(w, d, SHIFTS)
            alphas.append(alpha.requires_grad_(True))
            entries.append((K.AdaShiftPrep(w, beta, d, SHIFTS, 0), d, z, 2, False))
            gys.append(torch.randn_like(w))
            vals.append(torch.zeros(alpha.shape[0], device="cuda"))
            n += w.numel()
        regp = torch.tensor([0.1, 5.0], device="cuda")
        reg = (0.0, 0.0, vals, regp)

        def fwdbwd():
            for a in alphas:
                a.grad = None
            ys = K.adashift_prepared_multi(alphas, entries, False, reg=reg)
            torch.autograd.backward(list(ys), gys)

        f = t_ms(lambda: K.adashift_prepared_multi([a.detach() for a in alphas], entries, False))
        fb = t_ms(fwdbwd)
        out[name] = {"fwd_us": round(f * 1e3, 2), "bwd_us": round((fb - f) * 1e3, 2),
                     "fwd_gbs": round(12.0 * n / (f * 1e-3) / 1e9, 1),
                     "bwd_gbs": round(12.0 * n / ((fb - f) * 1e-3) / 1e9, 1)}
    print(json.dumps(out), flush=True)


def main():
    if "--blocks" in sys.argv:
        return blocks()
    torch.manual_seed(0)
    for shape in SHAPES:
        w = torch.randn(shape, device="cuda") * 0.05
        d, z, _ = K.scale_init(w, 2, False, True, "max")
        alpha, beta, _ = K.shift_init(w, d, SHIFTS)
        prep = K.AdaShiftPrep(w, beta, d, SHIFTS, 0)
        g = torch.randn_like(w)
        a = alpha.clone().requires_grad_(True)
        regp = torch.tensor([0.1, 5.0], device="cuda")
        vals = torch.zeros(alpha.shape[0], device="cuda")
        reg = (0.0, 0.0, vals, regp)

        def fwd_old():
            return K.adashift(alpha, beta, w, d, z, SHIFTS, 2, False, 0, 0)

        def fwd_new():
            return K.adashift_prepared(alpha, prep, d, z, 2, False, 0)

        y_old = K.AdaShiftFn.apply
        Co, Ci, kh, kw = shape

        def bwd_old():
            K.AdaShiftFn.backward(ctx_old, g)

        def bwd_new():
            K.AdaShiftPrepFn.backward(ctx_new, g)

        class Ctx:
            pass
        ctx_old = Ctx()
        ctx_old.saved_tensors = (alpha, beta, w, d, z)
        ctx_old.cfg = (tuple(SHIFTS), 2, False, False, False, reg)
        ctx_old.needs_input_grad = (True, False) + (False,) * 9
        ctx_new = Ctx()
        ctx_new.saved_tensors = (alpha, d, z)
        lo_hi = K.qrange(2, False)
        import ctypes as C
        ctx_new.cfg = (False, reg, [prep], ((C.c_int64 * 1)(Co), (C.c_int64 * 1)(Ci),
                                           (C.c_int64 * 1)(kh * kw), (C.c_int * 1)(lo_hi[0]),
                                           (C.c_int * 1)(lo_hi[1])))
        ctx_new.needs_input_grad = (False, True)
        n = w.numel()
        res = {"shape": shape, "elems": n}
        for name, fn in (("fwd_old", fwd_old), ("fwd_prep", fwd_new), ("bwd_old", bwd_old),
                         ("bwd_prep", bwd_new)):
            ms = t_ms(fn)
            res[name + "_us"] = round(ms * 1e3, 2)
            res[name + "_gbs"] = round(12.0 * n / (ms * 1e-3) / 1e9, 1)
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
