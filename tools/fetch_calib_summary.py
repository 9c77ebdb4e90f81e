"""FETCH_SIZE (KiB) per dispatch of tools/fetch_calib's three read widths against the 256 MB
each reads: the factor FETCH_SIZE * 1024 / bytes per width (0.5 = the guide's x2
correction applies).  python tools/fetch_calib_summary.py PMC_DIR"""
import collections
import csv
import glob
import json
import os
import statistics
import sys

files = glob.glob(os.path.join(sys.argv[1], "**", "*counter_collection.csv"), recursive=True)
vals = collections.defaultdict(float)
names = {}
for f in files:
    for r in csv.DictReader(open(f)):
        if r.get("Counter_Name") == "FETCH_SIZE":
            vals[(f, r["Dispatch_Id"])] += float(r["Counter_Value"])
            names[(f, r["Dispatch_Id"])] = r["Kernel_Name"]
by = collections.defaultdict(list)
for k, v in vals.items():
    n = names[k]
    if "read_w" not in n:
        continue
    w = "16B" if "4u>" in n else ("8B" if "2u>" in n else "4B")
    by[w].append(v)
out = {w: {"launches": len(v), "FETCH_SIZE_KiB_median": statistics.median(v),
           "fetch_over_bytes": round(statistics.median(v) * 1024 / (256 << 20), 4)}
       for w, v in sorted(by.items())}
print(json.dumps(out, indent=1))
