"""Durations of the bench step's full-size launches from a rocprofv3 kernel trace, for
comparison with the bench line's HIP-event kernel_ms: fq_fwd_pt_ride (the step: the A4
activation q/dq over 205.5 M elements with the 21 ResNet-18 weights' tiles riding on it)
and fq_fwd_pt (the activation alone), launches > 100 us.
    python tools/k1_trace_stats.py KERNEL_TRACE.csv"""
import csv
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import RESNET18_SHAPES  # noqa: E402

N_ACT = 1024 * 64 * 56 * 56
N_W = 0
for s in RESNET18_SHAPES:
    n = 1
    for d in s:
        n *= d
    N_W += n
rows = list(csv.DictReader(open(sys.argv[1])))
out = {}
for name, pat, elems in (("fq_fwd_pt_ride", "fq_fwd_pt_ride<", N_ACT + N_W),
                         ("fq_fwd_pt", "fq_fwd_pt<", N_ACT)):
    d = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rows if pat in r["Kernel_Name"]]
    big = sorted(v / 1e3 for v in d if v > 100e3)
    if not big:
        continue
    out[name] = {"launches": len(big), "avg_us": round(statistics.mean(big), 2),
                 "median_us": round(statistics.median(big), 2), "min_us": big[0], "max_us": big[-1],
                 "alg_bytes": 8 * elems,
                 "achieved_gbs_median": round(8.0 * elems / (statistics.median(big) * 1e-6) / 1e9, 1)}
print(json.dumps(out))
