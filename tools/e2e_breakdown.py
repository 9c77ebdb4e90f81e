"""Wall-time breakdown of a main_imagenet.py calibration run: every reconstruction call
(shifted-scale block recon, BRECQ block/layer recon) and every feature-cache pass is
timed with a device synchronize on both sides.  Arguments are main_imagenet.py's.
Prints one line per call and a per-kind summary."""
import collections
import importlib
import functools
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import main_imagenet  # noqa: E402
from shiftedscalequantization_amd import drivers as D  # noqa: E402
from shiftedscalequantization_amd.quant import block_recon as BR  # noqa: E402
from shiftedscalequantization_amd.quant import data_utils as DU  # noqa: E402

LF = importlib.import_module("shiftedscalequantization_amd.quant.layer_recon_fused_shiftedScale")
tot = collections.defaultdict(float)
cnt = collections.Counter()


def timed(kind, fn):
    @functools.wraps(fn)
    def w(*a, **k):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        r = fn(*a, **k)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        tot[kind] += dt
        cnt[kind] += 1
        print(f"[breakdown] {kind} #{cnt[kind]} {dt * 1e3:.1f} ms", flush=True)
        return r
    return w


BR._fast_loop = timed("brecq_loop", BR._fast_loop)
BR.save_inp_oup_data = timed("brecq_cache", BR.save_inp_oup_data)
D.cache_block_features = timed("shift_cache", D.cache_block_features)
D.block_recon_fused_shiftedScale = timed("shift_block_recon", D.block_recon_fused_shiftedScale)
LF._fused_loop = timed("shift_loop", LF._fused_loop)

t0 = time.perf_counter()
main_imagenet.main(sys.argv[1:])
torch.cuda.synchronize()
print(f"[breakdown] total {time.perf_counter() - t0:.2f} s")
for k in sorted(tot):
    print(f"[breakdown] {k:20s} {cnt[k]:4d} calls {tot[k]:8.2f} s")
