"""Focused A/B of the per-tensor q/dq kernel over launch geometries (grid, block,
unroll, chunked, cache policy), each against the float4 copy of the same tensor with
the same geometry; interleaved rounds in one process (cdna_hip_programming.md §5.4
rule 24).  Prints rows sorted by median q/dq GB/s."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from shiftedscalequantization_amd import kernels as K  # noqa: E402

dev = torch.device("cuda")
x = torch.empty(1024, 64, 56, 56, device=dev).normal_().relu_()
y = torch.empty_like(x)
d, z, _ = K.scale_init(x[:64], 4, False, False, "mse")
n = x.numel()
U = {1: 1, 2: 2, 4: 0, 8: 3, 16: 4}
B = {256: 0, 512: 1, 1024: 2}


def var(grid, block=256, unroll=4, chunked=0, pol=1, pipe=0):
    return pol | (U[unroll] << 4) | (grid << 8) | (chunked << 24) | (B[block] << 25) | (pipe << 27)


geoms = {}
for grid, block, unroll in ((256, 256, 8), (256, 256, 4), (512, 256, 4), (256, 512, 4)):
    for rcp in (0, 1):
        geoms[f"g{grid}b{block}u{unroll}{'_rcp' if rcp else '_ieee'}"] = var(grid, block, unroll) | (rcp << 27)


def t(fn, reps=20):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


res = {}
for rnd in range(5):
    for name, v in geoms.items():
        K.set_variant(v)
        res.setdefault((name, "fq"), []).append(8 * n / t(lambda: K.fake_quant_fwd(x, d, z, 4, out=y)) / 1e6)
        res.setdefault((name, "copy"), []).append(8 * n / t(lambda: K.stream_copy(x, y)) / 1e6)
K.set_variant(var(256))
rows = [{"geom": k[0], "kind": k[1], "variant": geoms[k[0]], "gbs_med": round(sorted(v)[len(v) // 2], 1),
         "gbs_min": round(min(v), 1)} for k, v in res.items()]
rows.sort(key=lambda r: -r["gbs_med"])
for r in rows:
    print(json.dumps(r))
