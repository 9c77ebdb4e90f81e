"""Per-iteration anatomy of the recon loop from a rocprofv3 kernel trace: finds the gather
launches (gather2_kernel, or gather_shift_fwd -- the fused iteration start -- one per
iteration), and for each iteration window sums kernel busy time by kernel family; reports
wall (gather-to-gather) vs GPU-busy time."""
import collections
import csv
import os
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
# iteration marker: the batch gather (default), or MARKER=<substring> (e.g. copyBuffer, the
# one index copy per iteration, when an iteration gathers several tensors)
MARK = os.environ.get("MARKER")


def is_mark(name):
    if MARK:
        return MARK in name
    return "gather2_kernel" in name or "gather_shift_fwd" in name


gi = [i for i, r in enumerate(rows) if is_mark(r["Kernel_Name"])]
# split into the two recon blocks by large gaps
segments, cur = [], [gi[0]]
for a, b in zip(gi, gi[1:]):
    if int(rows[b]["Start_Timestamp"]) - int(rows[a]["Start_Timestamp"]) > 5e6:
        segments.append(cur)
        cur = []
    cur.append(b)
segments.append(cur)


FULL = len(sys.argv) > 2 and sys.argv[2] == "full"


def fam(n):
    if FULL:
        return n[:200]
    n = n.split("(")[0]
    for k in ("ssq::", "igemm", "miopen", "batched_transpose", "at::native", "__amd", "Sub", "Op"):
        if k in n:
            return (n.replace("void ", "")[:60]) if k == "ssq::" else k
    return n[:40]


for seg in segments:
    seg = seg[30:-5]          # skip warm-up / tail
    if len(seg) < 10:
        continue
    t0, t1 = int(rows[seg[0]]["Start_Timestamp"]), int(rows[seg[-1]]["Start_Timestamp"])
    n_it = len(seg) - 1
    busy = collections.Counter()
    cnt = collections.Counter()
    for r in rows[seg[0]:seg[-1]]:
        d = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        busy[fam(r["Kernel_Name"])] += d
        cnt[fam(r["Kernel_Name"])] += 1
    wall = (t1 - t0) / n_it / 1e3
    tot = sum(busy.values()) / n_it / 1e3
    print(f"--- {n_it} iterations: wall {wall:.1f} us/iter, GPU busy {tot:.1f} us/iter, "
          f"{sum(cnt.values())/n_it:.1f} launches/iter")
    for k, v in busy.most_common(25):
        print(f"  {v/n_it/1e3:8.1f} us  x{cnt[k]/n_it:4.1f}  {k}")
