"""Anatomy of bench.py's q/dq step: device time (HIP events around a HIP-graph replay of
`reps` calls, so host launch cost is excluded) of the A4 act q/dq alone, the W2 weights
multi-segment q/dq alone, and the whole step, next to the eager step bench.py times.
usage: python tools/step_probe.py"""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from shiftedscalequantization_amd import kernels as K  # noqa: E402
from shiftedscalequantization_amd.recon_bench import graph_time_ms  # noqa: E402

dev = torch.device("cuda:0")
act, d_a, z_a, weights, dws, zws, bits = bench.make_workload(dev, 0, 1024)
y = torch.empty_like(act)
ys = [torch.empty_like(w) for w in weights]
n_w = sum(w.numel() for w in weights)


def act_only():
    K.fake_quant_fwd(act, d_a, z_a, 4, out=y)


def w_only():
    K.fake_quant_multi(weights, dws, zws, bits)


def step():
    act_only()
    w_only()


res = {"act_ms": graph_time_ms(act_only, reps=10), "weights_ms": graph_time_ms(w_only, reps=10),
       "step_graph_ms": graph_time_ms(step, reps=10)}
for _ in range(5):
    bench_step = lambda: (K.fake_quant_fwd(act, d_a, z_a, 4), K.fake_quant_multi(weights, dws, zws, bits))
    bench_step()
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(20):
    K.fake_quant_fwd(act, d_a, z_a, 4)
    K.fake_quant_multi(weights, dws, zws, bits)
torch.cuda.synchronize()
res["step_eager_ms"] = (time.perf_counter() - t0) / 20 * 1e3
res["weights_tb_s"] = 8.0 * n_w / (res["weights_ms"] * 1e-3) / 1e12
res["act_tb_s"] = 8.0 * act.numel() / (res["act_ms"] * 1e-3) / 1e12
res["weights_elems"] = n_w
print(json.dumps({k: round(v, 4) if isinstance(v, float) else v for k, v in res.items()}))
