"""HBM traffic per launch from two rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE are in
KiB and cannot share a pass on gfx950).  Per MI355X_MICROARCH.md §HBM, FETCH_SIZE reports
half the bytes of a wide coalesced streaming read on gfx950, so the read side is doubled:
    hbm_bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024
Usage: python tools/pmc_traffic.py <fetch_dir> <write_dir> <out.json>"""
import collections
import csv
import glob
import json
import os
import sys

KERNELS = {"fq_fwd_pt": "ssq::fq_fwd_pt<", "fq_fwd_pt_ride": "ssq::fq_fwd_pt_ride<",
           "fq_fwd_multi": "fq_fwd_multi_kernel", "stream_copy": "ssq::copy_kernel<"}


def per_dispatch(d, counter):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    vals = collections.defaultdict(float)
    names = {}
    for f in files:
        for r in csv.DictReader(open(f)):
            if r.get("Counter_Name") != counter:
                continue
            key = (f, r["Dispatch_Id"])
            vals[key] += float(r["Counter_Value"])
            names[key] = r["Kernel_Name"]
    out = collections.defaultdict(list)
    for k, v in vals.items():
        for tag, pat in KERNELS.items():
            if pat in names[k]:
                out[tag].append(v)
    return out


fetch = per_dispatch(sys.argv[1], "FETCH_SIZE")
write = per_dispatch(sys.argv[2], "WRITE_SIZE")
res = {}
for tag in KERNELS:
    if not fetch.get(tag) or not write.get(tag):
        continue
    f = sorted(fetch[tag])[len(fetch[tag]) // 2]
    w = sorted(write[tag])[len(write[tag]) // 2]
    res[tag] = {"launches": [len(fetch[tag]), len(write[tag])], "FETCH_SIZE_KiB_median": f,
                "WRITE_SIZE_KiB_median": w, "hbm_bytes_per_launch": (2.0 * f + w) * 1024.0,
                "correction": "read side doubled (gfx950 FETCH_SIZE = 1/2 of wide streaming reads)"}
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from shiftedscalequantization_amd.build import provenance  # noqa: E402
res["provenance"] = provenance()
json.dump(res, open(sys.argv[3], "w"), indent=1)
print(json.dumps(res, indent=1))
