"""Recon-iteration rate of one block of any architecture (block_recon_fused_shiftedScale,
batch 32, 1024-sample cache), the target of a rocprofv3 kernel trace (tools/trace_iter.py).
usage: python tools/block_anatomy.py ARCH BLOCK [iters] [deterministic 0/1]"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from shiftedscalequantization_amd.recon_bench import run_block  # noqa: E402

arch, name = sys.argv[1], sys.argv[2]
iters = int(sys.argv[3]) if len(sys.argv) > 3 else 100
det = bool(int(sys.argv[4])) if len(sys.argv) > 4 else False
n_cali = int(sys.argv[5]) if len(sys.argv) > 5 else 1024
torch.backends.cudnn.deterministic = det
torch.backends.cudnn.benchmark = not det
import time
t0 = time.time()
ips = run_block(torch.device("cuda"), name, iters=iters, warmup=10, arch=arch, n_cali=n_cali)
print(json.dumps({"arch": arch, "block": name, "deterministic": det, "iters_per_s": round(ips["ips"] if isinstance(ips, dict) else ips, 1),
                  "wall_s": round(time.time() - t0, 1)}), flush=True)
