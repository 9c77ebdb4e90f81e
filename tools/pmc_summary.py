"""Per-kernel PMC averages from a rocprofv3 --pmc run beside the same kernel's average
duration from a --kernel-trace run, with the derived figures of MI355X_MICROARCH.md's PMC
notes: effective clock = GRBM_GUI_ACTIVE / 8 XCDs / duration; MFMA-busy fraction =
SQ_VALU_MFMA_BUSY_CYCLES / (clock cycles x 1024 SIMDs); the wave-cycle buckets
(SQ_WAIT_ANY / SQ_WAIT_INST_ANY / SQ_ACTIVE_INST_ANY, quad-cycles) as fractions of
SQ_WAVE_CYCLES.
    python tools/pmc_summary.py PMC_DIR TRACE_DIR KERNEL_SUBSTRING"""
import collections
import csv
import glob
import os
import statistics
import sys


def _find(d, suffix):
    hits = glob.glob(os.path.join(d, "**", "*" + suffix), recursive=True)
    if not hits:
        raise SystemExit(f"no *{suffix} under {d}")
    return hits[0]


def main():
    pmc_dir, kt_dir, key = sys.argv[1:4]
    vals = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(_find(pmc_dir, "counter_collection.csv"))):
        if key in r["Kernel_Name"]:
            vals[r["Counter_Name"]][r.get("Dispatch_Id", r.get("Correlation_Id", ""))] += \
                float(r["Counter_Value"])
    avg = {c: statistics.mean(v.values()) for c, v in vals.items()}
    durs = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
            for r in csv.DictReader(open(_find(kt_dir, "kernel_trace.csv"))) if key in r["Kernel_Name"]]
    dur_ns = statistics.median(durs)
    print(f"kernel ~ {key}: {len(durs)} launches, median {dur_ns / 1e3:.2f} us")
    for c in sorted(avg):
        print(f"  {c:28s} {avg[c]:.4g}")
    if "GRBM_GUI_ACTIVE" in avg:
        cyc = avg["GRBM_GUI_ACTIVE"] / 8.0
        print(f"  effective clock            {cyc / dur_ns:.3f} GHz (GRBM_GUI_ACTIVE / 8 / trace "
              f"duration; the PMC run's own duration may differ)")
        if "SQ_VALU_MFMA_BUSY_CYCLES" in avg:
            print(f"  MFMA busy fraction         {avg['SQ_VALU_MFMA_BUSY_CYCLES'] / (cyc * 1024):.3f}")
    wc = avg.get("SQ_WAVE_CYCLES")
    if wc:
        for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS"):
            if c in avg:
                print(f"  {c:28s} {avg[c] / wc:.3f} of SQ_WAVE_CYCLES")


if __name__ == "__main__":
    main()
