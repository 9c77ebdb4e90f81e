"""Host-side cost of bench.py's step (argument checks, output allocation, table packing,
ctypes calls) beside its device time: if the host needs longer per step than the kernel,
the timed region measures the host.  python tools/step_host_time.py"""
import os
import statistics
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from shiftedscalequantization_amd import kernels as K  # noqa: E402
from shiftedscalequantization_amd.recon_bench import graph_time_ms  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    act, d_a, z_a, weights, dws, zws, bits = bench.make_workload(dev, 0, 1024)
    y_act = torch.empty_like(act)
    y_w = [torch.empty_like(w) for w in weights]
    plan = K.FqMultiPlan(weights, dws, zws, bits, out=y_w)
    mode = ["alloc"]

    def step():
        with K.deferred_fq_multi():
            if mode[0] == "plan":
                plan()
            else:
                K.fake_quant_multi(weights, dws, zws, bits, out=y_w if mode[0] == "out" else None)
            K.fake_quant_fwd(act, d_a, z_a, 4, out=y_act)

    for m in ("alloc", "out", "plan"):
        mode[0] = m
        for _ in range(20):
            step()
        torch.cuda.synchronize()
        host = []
        for _ in range(5):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(20):
                step()
            host.append((time.perf_counter() - t0) / 20 * 1e3)
            torch.cuda.synchronize()
        print(f"{m} (alloc: outputs per call, out: preallocated, plan: FqMultiPlan): host ms/step "
              f"(20 calls, no sync) median {statistics.median(host):.4f}  all "
              f"{[round(h, 4) for h in host]}")
    dev_ms = graph_time_ms(step, reps=20, rounds=5)
    print(f"device ms/step (graph replay): {dev_ms:.4f}")


if __name__ == "__main__":
    main()
