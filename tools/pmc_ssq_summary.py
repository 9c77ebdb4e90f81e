"""Per-kernel summary of rocprofv3 PMC passes over the ssq recon kernels: HBM bytes per
launch (FETCH_SIZE doubled per the gfx950 correction of MI355X_MICROARCH.md, + WRITE_SIZE;
both in KB) and the SQ busy counters.  usage: pmc_ssq_summary.py FETCH_DIR WRITE_DIR SQ_DIR"""
import collections
import csv
import glob
import json
import sys


def load(d):
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    n = collections.Counter()
    for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"]
            if "ssq" not in name and "prep" not in name:
                continue
            key = name.split("(")[0].replace("void ", "")
            agg[key][r["Counter_Name"]] += float(r["Counter_Value"])
            n[(key, r["Counter_Name"])] += 1
    return {k: {c: v / max(n[(k, c)], 1) for c, v in cs.items()} for k, cs in agg.items()}


fetch, write, sq = (load(d) for d in sys.argv[1:4])
out = {}
for k in sorted(set(fetch) | set(write) | set(sq)):
    e = {}
    if k in fetch:
        e["hbm_read_bytes_per_launch"] = 2 * 1024 * fetch[k].get("FETCH_SIZE", 0.0)
    if k in write:
        e["hbm_write_bytes_per_launch"] = 1024 * write[k].get("WRITE_SIZE", 0.0)
    if k in sq:
        e.update({c: round(v) for c, v in sq[k].items()})
        if sq[k].get("SQ_WAVE_CYCLES"):
            e["active_frac"] = round(sq[k].get("SQ_ACTIVE_INST_ANY", 0) / sq[k]["SQ_WAVE_CYCLES"], 3)
            e["valu_frac"] = round(sq[k].get("SQ_ACTIVE_INST_VALU", 0) / sq[k]["SQ_WAVE_CYCLES"], 3)
    out[k] = e
print(json.dumps(out, indent=1))
