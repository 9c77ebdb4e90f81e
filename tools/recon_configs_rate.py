"""iters/s of the BASELINE configs 3-5 loops (recon_bench.run_recon_configs, deterministic
solvers, batch 32), for A/B runs of a knob:

    python tools/recon_configs_rate.py [iters] [config ...]   e.g.  200 3 5"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from shiftedscalequantization_amd import recon_bench as RB  # noqa: E402


def main():
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    want = sys.argv[2:] or [c[0] for c in RB.RECON_CONFIGS]
    cfgs = tuple(c for c in RB.RECON_CONFIGS if c[0] in want)
    res = RB.run_recon_configs(torch.device("cuda", 0), 1, 0, iters=iters, configs=cfgs)
    print(json.dumps({k: v["iters_per_s"] for k, v in res.items()}), flush=True)


if __name__ == "__main__":
    main()
