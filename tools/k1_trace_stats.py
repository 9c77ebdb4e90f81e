"""Durations of the headline kernel's full-size launches (fq_fwd_pt over the 205.5 M
element activation: > 100 us) from a rocprofv3 kernel trace, for comparison with the bench
line's HIP-event kernel_ms.  usage: python tools/k1_trace_stats.py KERNEL_TRACE.csv"""
import csv
import json
import statistics
import sys

d = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in csv.DictReader(open(sys.argv[1]))
     if "fq_fwd_pt" in r["Kernel_Name"]]
big = sorted(v / 1e3 for v in d if v > 100e3)
alg = 8.0 * 1024 * 64 * 56 * 56
print(json.dumps({"kernel": "fq_fwd_pt", "launches": len(big), "avg_us": round(statistics.mean(big), 2),
                  "median_us": round(statistics.median(big), 2), "min_us": big[0], "max_us": big[-1],
                  "achieved_gbs_median": round(alg / (statistics.median(big) * 1e-6) / 1e9, 1)}))
