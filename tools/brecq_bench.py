"""BRECQ block_reconstruction iteration rate (ResNet-50 block_recon):
AdaRound weight phase and act-delta (LSQ) phase on one block, batch 32, synthetic data.
Rate = (T(iters_long) - T(iters_short)) / (iters_long - iters_short), so caching and setup
cancel out."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from shiftedscalequantization_amd import nets  # noqa: E402
from shiftedscalequantization_amd.quant import QuantModel, block_reconstruction  # noqa: E402


def build(arch, dev):
    torch.manual_seed(1005)
    qnn = QuantModel(nets.ARCHS[arch]().eval(), {"n_bits": 2, "channel_wise": True, "scale_method": "max"},
                     {"n_bits": 4, "channel_wise": False, "scale_method": "mse", "leaf_param": True})
    qnn.to(dev).eval()
    qnn.set_first_last_layer_to_8bit()
    return qnn


def block_of(qnn, path):
    m = qnn.model
    for part in path.split("."):
        m = m[int(part)] if part.isdigit() else getattr(m, part)
    return m


def timed(fn):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    fn()
    torch.cuda.synchronize()
    return time.perf_counter() - t0


def main():
    dev = torch.device("cuda")
    cali = torch.randn(128, 3, 224, 224, device=dev)
    res = {}
    for arch, path in (("resnet18", "layer1.0"), ("resnet50", "layer1.0")):
        for phase in ("weight", "act"):
            times = {}
            for iters in (20, 20, 220):      # the first run pays one-time setup (MIOpen)
                qnn = build(arch, dev)
                qnn.set_quant_state(True, phase == "act")
                with torch.no_grad():
                    qnn(cali[:64])
                blk = block_of(qnn, path)
                kw = dict(batch_size=32, iters=iters, weight=0.01, asym=True, b_range=(20, 2),
                          warmup=0.2, act_quant=phase == "act", opt_mode="mse")
                if phase == "act":
                    kw.update(lr=4e-4, p=2.4)
                times[iters] = timed(lambda: block_reconstruction(qnn, blk, cali, **kw))
            rate = 200 / (times[220] - times[20])
            res[f"{arch}.{path}.{phase}"] = round(rate, 1)
            print(json.dumps({"block": f"{arch}.{path}", "phase": phase, "iters_per_s": round(rate, 1)}),
                  flush=True)
    print(json.dumps({"brecq_iters_per_s": res}))


if __name__ == "__main__":
    main()
