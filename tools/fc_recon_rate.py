"""Iteration rate of the fc's AdaRound weight phase (main_imagenet.py:114-118:
layer_reconstruction on ResNet-18's last QuantModule, batch 32, synthetic data): the
end-to-end flow's 20000-iteration loop on a tiny layer, where the host's per-iteration work
can outlast the GPU's.  Rate = 2000 / (T(2200) - T(200)); then a cProfile of one
2200-iteration run (top host functions by own time).  Usage: python tools/fc_recon_rate.py"""
import cProfile
import io
import json
import os
import pstats
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from shiftedscalequantization_amd import nets  # noqa: E402
from shiftedscalequantization_amd.quant import QuantModel, QuantModule, layer_reconstruction  # noqa: E402


def build(dev):
    torch.manual_seed(1005)
    qnn = QuantModel(nets.ARCHS["resnet18"]().eval(), {"n_bits": 2, "channel_wise": True, "scale_method": "max"},
                     {"n_bits": 4, "channel_wise": False, "scale_method": "mse", "leaf_param": True})
    qnn.to(dev).eval()
    qnn.set_first_last_layer_to_8bit()
    return qnn


def run(dev, cali, iters):
    qnn = build(dev)
    qnn.set_quant_state(True, False)
    with torch.no_grad():
        qnn(cali[:64])
    fc = [m for m in qnn.modules() if isinstance(m, QuantModule)][-1]
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    layer_reconstruction(qnn, fc, cali, batch_size=32, iters=iters, weight=0.01, asym=True,
                         b_range=(20, 2), warmup=0.2, act_quant=False, opt_mode="mse")
    torch.cuda.synchronize()
    return time.perf_counter() - t0


def main():
    dev = torch.device("cuda")
    cali = torch.randn(256, 3, 224, 224, device=dev)
    run(dev, cali, 20)
    t = {n: run(dev, cali, n) for n in (200, 2200)}
    us = (t[2200] - t[200]) / 2000 * 1e6
    out = {"fc_adaround_us_per_iter": round(us, 2), "it_per_s": round(1e6 / us, 1)}
    print(json.dumps(out))
    # the chunk graph's own replay time (GPU work + launch boundaries, no host work between
    # iterations): 20 back-to-back replays of the loop's last chunk graph, HIP events
    from shiftedscalequantization_amd.quant import block_recon as BR
    BR.CHUNK_PROBE[0] = False
    run(dev, cali, 300)
    us_chunk = BR.CHUNK_PROBE[0]
    BR.CHUNK_PROBE[0] = None
    if us_chunk:
        print(json.dumps({"chunk_replay_us_per_iter": round(us_chunk, 2),
                          "iters_per_chunk": BR.CHUNK_ITERS}))
    pr = cProfile.Profile()
    pr.enable()
    run(dev, cali, 2200)
    pr.disable()
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(25)
    print(s.getvalue())


if __name__ == "__main__":
    main()
