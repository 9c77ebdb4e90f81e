"""Per-batch kernel breakdown of tools/val_profile.py's rocprofv3 kernel trace: the last
20 forwards (the timed batches) are located by their fc-layer epilogue launches... simpler:
every launch after the first timed batch's first conv is attributed to the timed region;
kernels are grouped by family and reported as us per batch.
    python tools/val_summary.py KERNEL_TRACE.csv [batches=20]"""
import collections
import csv
import sys


def family(n):
    if "bias_act_kernel" in n:
        return "K13 epilogue fwd (+A4 act q/dq)"
    if "fq_fwd_multi" in n or "fq_fwd_pt" in n or "fq_fwd" in n:
        return "K1 weight / act q/dq"
    if "igemm" in n or "miopen" in n.lower() or "conv" in n.lower() or "Cijk" in n or \
            "winograd" in n.lower() or "transpose" in n.lower() or "naive" in n.lower():
        return "MIOpen / rocBLAS conv"
    return n[:70]


def main():
    rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
    nb = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    # the timed batches are the last nb forwards: split on the first-layer conv of each
    # forward -- the launch that follows the previous forward's last (fc) launch; use the
    # count of launches per forward from the last nb * L launches
    total = len(rows)
    # launches per forward: the last forward ends at the last launch; find the period by the
    # name sequence of the final launches
    names = [r["Kernel_Name"] for r in rows]
    period = None
    for L in range(10, 400):
        if names[-L:] == names[-2 * L:-L] and names[-L:] == names[-3 * L:-2 * L]:
            period = L
            break
    if period is None:
        raise SystemExit("no periodic forward found")
    sel = rows[total - nb * period:]
    t0, t1 = int(sel[0]["Start_Timestamp"]), int(sel[-1]["End_Timestamp"])
    fam = collections.Counter()
    cnt = collections.Counter()
    for r in sel:
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        fam[family(r["Kernel_Name"])] += d
        cnt[family(r["Kernel_Name"])] += 1
    busy = sum(fam.values())
    print(f"launches per forward: {period}; wall per batch {(t1 - t0) / 1e3 / nb:.1f} us, "
          f"GPU busy {busy / nb:.1f} us")
    for k, v in fam.most_common():
        print(f"  {v / nb:8.1f} us  x{cnt[k] / nb:5.1f}  {k}")
    per = collections.Counter()
    pcnt = collections.Counter()
    for r in sel:
        per[r["Kernel_Name"][:100]] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        pcnt[r["Kernel_Name"][:100]] += 1
    print("per kernel (us per batch, launches per batch):")
    for k, v in per.most_common(25):
        print(f"  {v / nb:8.1f} us  x{pcnt[k] / nb:5.1f}  {k}")


if __name__ == "__main__":
    main()
