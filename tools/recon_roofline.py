"""SURVEY §8(d) reconstruction roofline from a rocprofv3 kernel trace of the REAL loop.

    python tools/recon_roofline.py KERNEL_TRACE.csv [OUT.json]

The trace is that of `bench.py` (recon_bench.run_recon_bench: for every ResNet-18 block
one deterministic-solver loop, then one benchmark-solver loop; 20 warm-up + K timed
iterations each, batch 32, bias_cal).  Loop segments are found from the gather launches
(one per iteration; segments split at > 5 ms gaps); the deterministic loop of block b is
the (2b)-th segment.  Over its timed iterations every launch is classified by kernel name
and priced with the algorithmic bytes of that launch (A = batch * C_out * H' * W' output
elements of the block's convs, N_W its weights, N_in its gathered input elements):

  K5p  shift_fwd_prep                        12 B / weight   (packed floors + h(beta) in, W^ out)
  K6p  alpha_bwd_prep (+ _stage2)            12 B / weight   (dL/dW^ + packed floors + h(beta) in)
  K14  gather2_kernel                         8 B / input elem (batch rows in and out)
  K14+K5p gather_shift_fwd                    8 B / input elem + 12 B / weight (the two above
                                              in one launch: the iteration start)
  K13  bias_act_kernel<RES,...>              (8 + 4 RES) B / A (y [+ residual] in, activation out)
  K13b epilogue_bwd_rows<RES,...,LOSS=false> (12 + 4 RES + 4 GRES) B / A (g, y [, res] in,
                                              gy [, g_res] out)
  K11t epilogue_bwd_rows<...,LOSS=true>      (12 + 4 RES + 4 GRES) B / A, the fused tail: y,
                                              target rows [, res] in, gy [, g_res] out
  K11  lp_loss_kernel                         12 B / A (prediction, target rows in, gradient out)
  K12  adam_kernel                            28 B / parameter (p, g, m, v in; p, m, v out);
                                              at world 1 the step rides on K6p's launch
                                              (ssq_adam_arm) and its bytes are priced there

GRES (a residual gradient is written) holds for blocks with a downsample branch.  Every
other launch (MIOpen / hipBLASLt convs, the K17 / GEMM-operand conv kernels) is reported
as conv time, outside the HBM set.  Writes the JSON that bench.py reports as
`roofline_recon` (profiles/<round>_recon_roofline.json)."""
import collections
import csv
import json
import os
import re
import sys

BATCH = 32
S = 3
# ResNet-18 blocks (models/resnet.py:260): input (C_in, H, W) at 224x224, C_out, stride
BLOCKS = {"layer1.0": ((64, 56, 56), 64, 1), "layer1.1": ((64, 56, 56), 64, 1),
          "layer2.0": ((64, 56, 56), 128, 2), "layer2.1": ((128, 28, 28), 128, 1),
          "layer3.0": ((128, 28, 28), 256, 2), "layer3.1": ((256, 14, 14), 256, 1),
          "layer4.0": ((256, 14, 14), 512, 2), "layer4.1": ((512, 7, 7), 512, 1)}
HBM_PEAK_GBS = 8000.0


def block_sizes(name):
    (cin, h, w), cout, stride = BLOCKS[name]
    ho, wo = (h + 2 - 3) // stride + 1, (w + 2 - 3) // stride + 1
    ds = stride != 1 or cin != cout
    n_w = cout * cin * 9 + cout * cout * 9 + (cout * cin if ds else 0)
    # alpha rows = input channels per conv; bias_cal adds gamma^z / phi^z per output channel
    n_par = (cin + cout + (cin if ds else 0)) * S + 2 * cout * (3 if ds else 2)
    return {"A": BATCH * cout * ho * wo, "N_W": n_w, "N_in": BATCH * cin * h * w, "ds": ds,
            "n_params": n_par}


def targs(name):
    m = re.search(r"<([^>]*)>", name)
    if not m:
        return []
    return [a.strip() for a in m.group(1).split(",")]


def classify(name, sz):
    """(class, algorithmic bytes) of one launch, or (None, 0) outside the HBM set."""
    a = targs(name)
    A = sz["A"]
    if "gather_shift_fwd" in name:
        return "K14_K5p_gather_adashift_fwd", 8 * sz["N_in"] + 12 * sz["N_W"]
    if "shift_fwd_prep" in name:
        return "K5p_adashift_fwd", 12 * sz["N_W"]
    if "alpha_bwd_prep_stage2" in name:
        return "K6p_adashift_bwd", 0
    if "alpha_bwd_prep" in name:
        return "K6p_adashift_bwd", 12 * sz["N_W"]
    if "gather2_kernel" in name:
        return "K14_gather", 8 * sz["N_in"]
    if "bias_act_kernel" in name:
        res = a[0] == "true"
        return "K13_epilogue_fwd", (8 + 4 * res) * A
    if "epilogue_bwd_rows" in name:
        # RES / LOSS print as bool or int (LOSS: 0 none, 1 p = 2, 2 general p; RES 2: the
        # downsample's epilogue folded in -- the same bytes, its raw output in place of res)
        res, loss = a[0] not in ("false", "0"), a[5] not in ("false", "0")
        gres = res and sz["ds"]
        b = (12 + 4 * res + 4 * gres) * A
        return ("K11t_fused_tail" if loss else "K13b_epilogue_bwd"), b
    if "lp_loss_kernel" in name:
        return "K11_lp_loss", 12 * A
    if "adam_kernel" in name:
        return "K12_adam", 28 * sz["n_params"]
    return None, 0


def segments(rows):
    gi = [i for i, r in enumerate(rows) if "gather2_kernel" in r["Kernel_Name"] or
          "gather_shift_fwd" in r["Kernel_Name"]]
    segs, cur = [], [gi[0]]
    for a, b in zip(gi, gi[1:]):
        if int(rows[b]["Start_Timestamp"]) - int(rows[a]["Start_Timestamp"]) > 5e6:
            segs.append(cur)
            cur = []
        cur.append(b)
    segs.append(cur)
    return [s for s in segs if len(s) >= 50]          # the loops (not one-off gathers)


def analyse(path, warmup=20):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    segs = segments(rows)
    names = list(BLOCKS)
    if len(segs) != 2 * len(names):
        raise SystemExit(f"expected {2 * len(names)} loop segments, found {len(segs)}")
    out, tot_b, tot_us = {}, 0.0, 0.0
    for b, name in enumerate(names):
        seg = segs[2 * b][warmup:]          # the timed iterations of the deterministic loop
        sz = block_sizes(name)
        n_it = len(seg) - 1
        us, by, cnt = collections.Counter(), collections.Counter(), collections.Counter()
        other_us = 0.0
        for r in rows[seg[0]:seg[-1]]:
            d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
            cls, nb = classify(r["Kernel_Name"], sz)
            if cls is None:
                other_us += d
                continue
            us[cls] += d
            by[cls] += nb
            cnt[cls] += 1
        if not cnt["K12_adam"]:
            # the optimizer step rides on the alpha backward's launch (ssq_adam_arm): its
            # 28 B / parameter are that launch's too
            by["K6p_adashift_bwd"] += 28 * sz["n_params"] * n_it
        t0, t1 = int(rows[seg[0]]["Start_Timestamp"]), int(rows[seg[-1]]["Start_Timestamp"])
        cls_out = {c: {"us": round(us[c] / n_it, 2), "bytes": int(by[c] / n_it),
                       "launches": round(cnt[c] / n_it, 2),
                       "gbs": round(by[c] / (us[c] * 1e-6) / 1e9, 1) if us[c] else None}
                   for c in sorted(us)}
        b_it, us_it = sum(by.values()) / n_it, sum(us.values()) / n_it
        out[name] = {"iterations": n_it, "wall_us": round((t1 - t0) / 1e3 / n_it, 2),
                     "hbm_set_us": round(us_it, 2), "hbm_set_bytes": int(b_it),
                     "achieved_gbs": round(b_it / (us_it * 1e-6) / 1e9, 1),
                     "other_us": round(other_us / n_it, 2), "kernels": cls_out, "sizes": sz}
        tot_b += b_it
        tot_us += us_it
    ach = tot_b / (tot_us * 1e-6) / 1e9
    return {"bound": "hbm", "source": "rocprofv3 --kernel-trace of bench.py's recon loops "
                                      "(deterministic solvers, timed iterations)",
            "kernels": "K5p + K6p + K11t fused tail / K11 + K13 epilogues + K14 gather + "
                       "K12 adam, every launch of the loop iteration, all 8 blocks",
            "bytes_per_iteration": int(tot_b), "us_per_iteration": round(tot_us, 2),
            "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(ach / HBM_PEAK_GBS, 4), "blocks": out}


def _short(name):
    n = name.split("(")[0]
    n = n.replace("void ", "").replace("ssq::", "")
    return n[:60]


def analyse_configs(trace, side_path):
    """BASELINE configs 3-5 (tools/recon_configs_trace.py): each timed region lies between two
    marker launches (write_probe); its ssq-set launches (tools/ssq_bytes.ssq_kernel) are timed
    from the trace, and priced with the algorithmic bytes of the entry points one iteration
    calls (the side file's ledger, from the iteration the loop captured and replays)."""
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    import ssq_bytes
    side = json.load(open(side_path))
    rows = list(csv.DictReader(open(trace)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    marks = [i for i, r in enumerate(rows) if "write_probe" in r["Kernel_Name"]]
    pairs = list(zip(marks[0::2], marks[1::2]))
    regions = side["regions"]
    if len(pairs) != len(regions):
        raise SystemExit(f"expected {len(regions)} marked regions, found {len(pairs)}")
    out, tot_b, tot_us = {}, 0.0, 0.0
    for (a, b), reg in zip(pairs, regions):
        n_it = reg["iterations"]
        us, cnt, conv_us, other_us = collections.Counter(), collections.Counter(), 0.0, 0.0
        for r in rows[a + 1:b]:
            d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
            name = r["Kernel_Name"]
            if ssq_bytes.ssq_kernel(name):
                us[_short(name)] += d
                cnt[_short(name)] += 1
            elif "ssq::" in name or "wgrad_gemm_operands" in name:
                conv_us += d
            else:
                other_us += d
        wall = (int(rows[b]["Start_Timestamp"]) - int(rows[a]["End_Timestamp"])) / 1e3
        ssq_us = sum(us.values()) / n_it
        by = reg["bytes_per_iteration"]
        key = reg["config"] + ("" if reg["phase"] == "fused_loop" else "_" + reg["phase"])
        out[key] = {
            "arch": reg["arch"], "block": reg["block"], "phase": reg["phase"], "iterations": n_it,
            "wall_us_per_iteration": round(wall / n_it, 1),
            "ssq_set_us": round(ssq_us, 2), "ssq_set_bytes": int(by),
            "achieved": round(by / (ssq_us * 1e-6) / 1e9, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(by / (ssq_us * 1e-6) / 1e9 / HBM_PEAK_GBS, 4),
            "conv_side_ssq_kernels_us": round(conv_us / n_it, 1),
            "library_convs_gemms_other_us": round(other_us / n_it, 1),
            "kernels": {k: {"us": round(v / n_it, 2), "launches": round(cnt[k] / n_it, 2)}
                        for k, v in us.most_common()},
            "ledger": reg["ledger"]}
        tot_b += by
        tot_us += ssq_us
    return {"bound": "hbm", "source": "rocprofv3 --kernel-trace of tools/recon_configs_trace.py "
                                      "(configs 3-5's loops, deterministic solvers, timed iterations)",
            "kernels": "every ssq:: launch of the loop iteration except conv arithmetic (K17 weight "
                       "gradients, K18 depthwise convs, im2col operands); bytes: the iteration's "
                       "entry points' operands (tools/ssq_bytes.py)",
            "configs": out}


if __name__ == "__main__" and sys.argv[1] == "--configs":
    res = analyse_configs(sys.argv[2], sys.argv[3])
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from shiftedscalequantization_amd.build import provenance
    res["provenance"] = provenance()
    with open(sys.argv[4], "w") as f:
        f.write(json.dumps(res, indent=1) + "\n")
    for k, v in res["configs"].items():
        print(f"{k} {v['arch']} {v['block']} {v['phase']}: wall {v['wall_us_per_iteration']} us/it, "
              f"ssq set {v['ssq_set_us']} us {v['ssq_set_bytes'] / 1e6:.2f} MB = {v['achieved']} GB/s "
              f"({v['frac']}), conv-side ssq {v['conv_side_ssq_kernels_us']} us, library/other "
              f"{v['library_convs_gemms_other_us']} us")
        for c, kk in v["kernels"].items():
            print(f"    {c:60s} {kk['us']:8.2f} us x{kk['launches']}")
    sys.exit(0)

if __name__ == "__main__":
    res = analyse(sys.argv[1])
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from shiftedscalequantization_amd.build import provenance
    res["provenance"] = provenance()
    txt = json.dumps(res, indent=1)
    if len(sys.argv) > 2:
        with open(sys.argv[2], "w") as f:
            f.write(txt + "\n")
    print(json.dumps({k: v for k, v in res.items() if k != "blocks"}))
    for name, v in res["blocks"].items():
        print(f"{name}: {v['hbm_set_us']:7.2f} us {v['hbm_set_bytes'] / 1e6:7.2f} MB "
              f"{v['achieved_gbs']:7.1f} GB/s  (other {v['other_us']:.1f} us, wall {v['wall_us']:.1f})")
        for c, k in v["kernels"].items():
            print(f"    {c:20s} {k['us']:7.2f} us x{k['launches']:.0f} {k['bytes'] / 1e6:7.2f} MB {k['gbs']}")
