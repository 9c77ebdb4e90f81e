"""Focused A/B of the per-tensor q/dq kernel: division form (div_rn vs IEEE divide) x a
few launch geometries, against the float4 copy of the same tensor; interleaved rounds in
one process (cdna_hip_programming.md §5.4 rule 24).  Also checks that both division
forms give bit-identical outputs on the full tensor."""
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
IEEE = 1 << 27
base = 1 | (256 << 8)                       # NT, unroll 4, grid 256, block 256

# bit-identical check
K.set_variant(base)
a = K.fake_quant_fwd(x, d, z, 4)[0]
K.set_variant(base | IEEE)
b = K.fake_quant_fwd(x, d, z, 4)[0]
torch.cuda.synchronize()
same = bool(torch.equal(a.view(torch.int32), b.view(torch.int32)))
print(json.dumps({"bit_identical_div_rn_vs_ieee": same}))
assert same


def t(fn, reps=20):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


geoms = {"g256b256": 1 | (256 << 8), "g512b256": 1 | (512 << 8), "g1024b256": 1 | (1024 << 8),
         "g512b512": 1 | (512 << 8) | (1 << 25), "g256b1024ch": 1 | (256 << 8) | (1 << 24) | (2 << 25),
         "g1024b1024ch": 1 | (1024 << 8) | (1 << 24) | (2 << 25),
         "g2048b256u2": 1 | (2 << 4) | (2048 << 8), "g256b256u8": 1 | (3 << 4) | (256 << 8)}
res = {}
for rnd in range(5):
    for name, v in geoms.items():
        for div in ("rn", "ieee"):
            K.set_variant(v | (IEEE if div == "ieee" else 0))
            res.setdefault((name, div), []).append(8 * n / t(lambda: K.fake_quant_fwd(x, d, z, 4, out=y)) / 1e6)
        K.set_variant(v)
        res.setdefault((name, "copy"), []).append(8 * n / t(lambda: K.stream_copy(x, y)) / 1e6)
K.set_variant(base)
rows = [{"geom": k[0], "kind": k[1], "gbs_med": round(sorted(v)[len(v) // 2], 1),
         "gbs_max": round(max(v), 1)} for k, v in res.items()]
rows.sort(key=lambda r: -r["gbs_med"])
for r in rows:
    print(json.dumps(r))
