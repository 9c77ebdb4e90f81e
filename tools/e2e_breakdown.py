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

_marks = {}


def _hook(i, iters):
    """Per-phase times of each BRECQ device loop: setup (entry .. i=0), eager warm-up
    (0-3), capture + first replay (3-4), replays 4-20, steady state 20 .. iters-1, the last
    iteration (iters-1 .. end)."""
    if i in (-1, 0, 3, 4, 20, iters - 1, iters):
        torch.cuda.synchronize()
        _marks[i] = time.perf_counter()
        if i == iters and 20 in _marks:
            m = _marks
            print(f"[breakdown] brecq setup {1e3 * (m[0] - m[-1]):.1f} ms, warmup {1e3 * (m[3] - m[0]):.1f} ms, "
                  f"capture {1e3 * (m[4] - m[3]):.1f} ms, 4-20 {1e3 * (m[20] - m[4]):.1f} ms, "
                  f"steady {1e6 * (m[iters - 1] - m[20]) / (iters - 21):.1f} us/iter, "
                  f"last {1e3 * (m[iters] - m[iters - 1]):.1f} ms", flush=True)
            _marks.clear()


# the per-iteration hook turns the loops' chunked graph replays off (block_recon.ChunkGraph
# needs ITER_HOOK unset): SSQ_BREAKDOWN_HOOK=0 keeps the per-call times only
if os.environ.get("SSQ_BREAKDOWN_HOOK", "1") != "0":
    BR.ITER_HOOK = _hook
t0 = time.perf_counter()
main_imagenet.main(sys.argv[1:])
torch.cuda.synchronize()
print(f"[breakdown] total {time.perf_counter() - t0:.2f} s")
for k in sorted(tot):
    print(f"[breakdown] {k:20s} {cnt[k]:4d} calls {tot[k]:8.2f} s")
