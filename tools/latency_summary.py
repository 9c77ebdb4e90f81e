"""Summary of tools/latency_probe's rocprofv3 kernel trace: per (grid, kernel, cold|hot)
the median launch duration in us (launch order: per grid, 50 cold rounds of
empty / chain1 / chain2 / chain3 [/ wide16] each after a 1 GB copy, then 50 hot rounds of
chain1 / chain2 back to back)."""
import csv
import statistics
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
rows = [r for r in rows if "k_flush" not in r["Kernel_Name"] and "k_" in r["Kernel_Name"]]
out, i = [], 0
for grid in (1, 16, 256, 1024):
    names = ["k_empty", "k_chain1", "k_chain2", "k_chain3"] + (["k_wide16"] if grid <= 256 else [])
    d = {n: [] for n in names}
    for _ in range(50):
        for n in names:
            assert n in rows[i]["Kernel_Name"], (n, rows[i]["Kernel_Name"])
            d[n].append((int(rows[i]["End_Timestamp"]) - int(rows[i]["Start_Timestamp"])) / 1e3)
            i += 1
    h = {"k_chain1": [], "k_chain2": []}
    for _ in range(50):
        for n in h:
            h[n].append((int(rows[i]["End_Timestamp"]) - int(rows[i]["Start_Timestamp"])) / 1e3)
            i += 1
    for n, v in d.items():
        print(f"grid {grid:5d} cold {n:9s} median {statistics.median(v):7.2f} us")
    for n, v in h.items():
        print(f"grid {grid:5d} hot  {n:9s} median {statistics.median(v):7.2f} us")

# after-probe: k_empty after each of the five producers, 50 rounds
names = ["512MB copy", "512MB copy, nt stores", "512MB read-only", "8MB copy", "64MB copy"]
d = {n: [] for n in names}
for _ in range(50):
    for n in names:
        assert "k_empty" in rows[i]["Kernel_Name"], rows[i]["Kernel_Name"]
        d[n].append((int(rows[i]["End_Timestamp"]) - int(rows[i]["Start_Timestamp"])) / 1e3)
        i += 1
for n, v in d.items():
    print(f"empty kernel after {n:22s} median {statistics.median(v):7.2f} us")
