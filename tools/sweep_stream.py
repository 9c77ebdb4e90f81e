"""A/B sweep of the streaming q/dq + copy kernels (cache policy x unroll x grid),
interleaved rounds in one process (cdna_hip_programming.md §5.4 rule 24)."""
import itertools
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from shiftedscalequantization_amd import kernels as K  # noqa: E402

dev = torch.device("cuda")
x = torch.empty(1024, 64, 56, 56, device=dev).normal_().relu_()
y = torch.empty_like(x)
d, z = torch.tensor(0.3, device=dev), torch.tensor(0.0, device=dev)
n = x.numel()


def t(fn, reps=10):
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


variants = []
for pol, un, grid, ch, blk in itertools.product([0, 1, 3], [1, 2, 0], [256, 512, 768, 1024],
                                                [0, 1], [0, 1, 2]):
    variants.append(pol | (un << 4) | (grid << 8) | (ch << 24) | (blk << 25))
res = {v: {"fq": [], "copy": []} for v in variants}
for rnd in range(3):
    for v in variants:
        K.set_variant(v)
        res[v]["fq"].append(8 * n / t(lambda: K.fake_quant_fwd(x, d, z, 4)) / 1e6)
        res[v]["copy"].append(8 * n / t(lambda: K.stream_copy(x, y)) / 1e6)
rows = []
for v in variants:
    rows.append({"variant": v, "policy": v & 3, "unroll": {0: 4, 1: 1, 2: 2, 3: 8}[(v >> 4) & 15],
                 "grid": (v >> 8) & 0xFFFF, "chunked": (v >> 24) & 1,
                 "block": {0: 256, 1: 512, 2: 1024}[(v >> 25) & 3],
                 "fq_gbs_med": sorted(res[v]["fq"])[1],
                 "copy_gbs_med": sorted(res[v]["copy"])[1]})
rows.sort(key=lambda r: -r["fq_gbs_med"])
for r in rows[:25]:
    print(json.dumps(r))
print("best copy:", json.dumps(max(rows, key=lambda r: r["copy_gbs_med"])))
