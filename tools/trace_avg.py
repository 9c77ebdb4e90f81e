"""Per-kernel launch count and average / median duration (us) from a rocprofv3
kernel_trace.csv, in order of first appearance; optional name filter substrings.
    python tools/trace_avg.py KERNEL_TRACE.csv [substr ...] [--groups=G]
--groups=G splits each kernel's launches into G consecutive equal groups (e.g. the blocks
of tools/alpha_cold.py, in order)."""
import collections
import csv
import statistics
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    keys = [k for k in sys.argv[2:] if not k.startswith("--groups=")]
    groups = [int(k.split("=")[1]) for k in sys.argv[2:] if k.startswith("--groups=")]
    groups = groups[0] if groups else 1
    dur = collections.OrderedDict()
    for r in rows:
        n = r["Kernel_Name"]
        if keys and not any(k in n for k in keys):
            continue
        dur.setdefault(n[:90], []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    for n, v in dur.items():
        per = len(v) // groups
        for gi in range(groups):
            w = v[gi * per:(gi + 1) * per] if groups > 1 else v
            tag = f"[{gi}] " if groups > 1 else ""
            print(f"{len(w):6d}  avg {sum(w) / len(w):8.2f}  med {statistics.median(w):8.2f}  {tag}{n}")


if __name__ == "__main__":
    main()
