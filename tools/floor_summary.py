"""Summary of tools/floor_probe's rocprofv3 kernel trace: every k_empty launch's own
duration (begin..end) and the gap from the end of the kernel before it to its begin,
labelled by the probe's launch order (floor_probe.hip: policy plain / nt / sc1 x dirty MB
0 / 4 / 16 / 64 x reps after a producer; then empty after empty; then the graph pairs),
median over the repetitions."""
import csv
import statistics
import sys

REPS = 30
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
labels = [f"{pol:5s} dirty {mb:2d} MB" for pol in ("plain", "nt", "sc1") for mb in (0, 4, 16, 64)
          for _ in range(REPS)]
labels += ["empty after evict"] * 0
seq = []
for prev, cur in zip(rows, rows[1:]):
    if "k_empty" in cur["Kernel_Name"]:
        seq.append((prev["Kernel_Name"].split("(")[0],
                    (int(cur["End_Timestamp"]) - int(cur["Start_Timestamp"])) / 1e3,
                    (int(cur["Start_Timestamp"]) - int(prev["End_Timestamp"])) / 1e3))
out = {}
i = 0
for lab in labels:
    out.setdefault(lab, []).append(seq[i])
    i += 1
# empty + empty: per rep, the first follows the evict pass, the second the first
for _ in range(REPS):
    out.setdefault("empty after evict (no producer)", []).append(seq[i])
    out.setdefault("empty after empty", []).append(seq[i + 1])
    i += 2
for pol in ("plain", "nt", "sc1"):
    for _ in range(REPS):
        out.setdefault(f"{pol:5s} dirty 16 MB (graph)", []).append(seq[i])
        i += 1
for lab, v in out.items():
    print(f"{lab:34s} after {v[0][0]:28s} n={len(v):3d} empty_dur_med={statistics.median(x[1] for x in v):6.2f} us "
          f"gap_before_med={statistics.median(x[2] for x in v):6.2f} us")
print(f"# {i} of {len(seq)} k_empty launches labelled")
