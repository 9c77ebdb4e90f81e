"""BASELINE configs 3-5's reconstruction loops (recon_bench.run_recon_configs) with a marker
kernel (ssq_stream_probe's write_probe on 64 floats, a launch no loop makes) at the start and
the end of every timed region, for rocprofv3:

    rocprofv3 --kernel-trace --output-format csv -d DIR -o cfg -- \
        python3 tools/recon_configs_trace.py [iters] SIDE.json

SIDE.json lists the regions in order (config, phase, timed iterations); tools/recon_roofline.py
--configs prices each region's ssq launches from the trace."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import torch  # noqa: E402

from shiftedscalequantization_amd import kernels as K, recon_bench as RB  # noqa: E402


def main():
    iters = int(sys.argv[1]) if len(sys.argv) > 2 else 100
    side = sys.argv[-1]
    dev = torch.device("cuda", 0)
    buf = torch.zeros(64, device=dev)
    regions = []

    def mark(n):
        K.stream_write(buf)
        torch.cuda.synchronize(dev)
        if n is not None:
            regions.append(n)

    # the ledger: the algorithmic bytes of every entry point called while the loop captures
    # its single-iteration graph (iteration GRAPH_WARMUP: the iteration every replay runs)
    from shiftedscalequantization_amd import _capi as A
    from shiftedscalequantization_amd.quant import block_recon as BRm
    import ssq_bytes
    cur, ledgers = {"loop": -1, "i": -1}, []

    def note(i):
        if i == 0:
            cur["loop"] += 1
            ledgers.append({})
        cur["i"] = i

    def on_call(name, args):
        if cur["i"] == BRm.GRAPH_WARMUP and cur["loop"] >= 0:
            b = ssq_bytes.bytes_of(name, args)
            if b is not None:
                led = ledgers[cur["loop"]]
                n, tot = led.get(name, (0, 0))
                led[name] = (n + 1, tot + b)

    RB.MARK[0], RB.ITER_NOTE[0], A.CALL_HOOK = mark, note, on_call
    try:
        res = RB.run_recon_configs(dev, 1, 0, iters=iters)
    finally:
        RB.MARK[0], RB.ITER_NOTE[0], A.CALL_HOOK = None, None, None
    order = []
    for cfg, arch, name, loop in RB.RECON_CONFIGS:
        for ph in (("weight_phase", "act_phase") if loop == "brecq" else ("fused_loop",)):
            order.append({"config": f"config{cfg}", "arch": arch, "block": name, "phase": ph})
    assert len(order) == len(regions) == len(ledgers), (order, regions, len(ledgers))
    for o, n, led in zip(order, regions, ledgers):
        o["iterations"] = n
        o["ledger"] = {k: {"calls": c, "bytes": b} for k, (c, b) in sorted(led.items())}
        o["bytes_per_iteration"] = sum(b for _, b in led.values())
    json.dump({"regions": order, "result": res}, open(side, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
