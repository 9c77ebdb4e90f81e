"""BRECQ's act phase on ResNet-18 blocks (the --bias_cal flow's act phase: fused K13 epilogues
with the act quantizer, the fused tail at p = 2.4) timed on the production loop, for A/Bs of
the act-quant epilogue kernels (e.g. SSQ_EPI_FASTDIV=0 / 1, read once per process):

    SSQ_EPI_FASTDIV=1 python tools/act_ab.py [iters] [blocks...]

Prints one JSON line: iterations per second per block (deterministic solvers, batch 32 of
1024 synthetic calibration images' block features, timed from the first chunk replay at or
after 20 iterations) and the act deltas reached (identical across bit-identical variants)."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from shiftedscalequantization_amd import nets  # noqa: E402
from shiftedscalequantization_amd.quant import QuantModel, block_recon as BR  # noqa: E402
from shiftedscalequantization_amd.quant import block_reconstruction  # noqa: E402
from shiftedscalequantization_amd.recon_bench import _block  # noqa: E402


def main():
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 300
    blocks = sys.argv[2:] or ["layer1.0", "layer4.0"]
    torch.backends.cudnn.benchmark, torch.backends.cudnn.deterministic = False, True
    dev = torch.device("cuda", 0)
    torch.manual_seed(1005)
    qnn = QuantModel(nets.resnet18().eval().to(dev),
                     {"n_bits": 2, "channel_wise": True, "scale_method": "max"},
                     {"n_bits": 4, "channel_wise": False, "scale_method": "mse", "leaf_param": True})
    qnn.to(dev).eval()
    qnn.set_first_last_layer_to_8bit()
    g = torch.Generator(device=dev).manual_seed(1005)
    cali = torch.empty(1024, 3, 224, 224, device=dev).normal_(generator=g)
    qnn.set_quant_state(True, True)
    with torch.no_grad():
        qnn(cali[:64])
    # gamma^z / phi^z off the identity, as after a --bias_cal weight phase
    gen = torch.Generator().manual_seed(7)
    for m in qnn.modules():
        if hasattr(m, "alpha_out"):
            with torch.no_grad():
                m.alpha_out.copy_(1 + 0.05 * torch.randn(m.alpha_out.shape, generator=gen))
                m.beta_out.copy_(0.02 * torch.randn(m.beta_out.shape, generator=gen))
    qnn.disable_network_output_quantization()
    out = {"fastdiv": os.environ.get("SSQ_EPI_FASTDIV", "default"), "iters_per_s": {},
           "deltas": {}}
    total, warm = iters + 20, 20
    for name in blocks:
        block = _block(qnn, name)
        st = {}

        def hook(i):
            if "t0" not in st and i >= warm:
                torch.cuda.synchronize(dev)
                st["t0"], st["i0"] = time.perf_counter(), i
            elif i == total and "t0" in st:
                torch.cuda.synchronize(dev)
                st["t1"] = time.perf_counter()

        BR.TIMING_HOOK = hook
        try:
            torch.manual_seed(1005)
            block_reconstruction(qnn, block, cali, batch_size=32, iters=total, act_quant=True,
                                 opt_mode="mse", lr=4e-4, p=2.4)
        finally:
            BR.TIMING_HOOK = None
        out["iters_per_s"][name] = round((total - st["i0"]) / (st["t1"] - st["t0"]), 2)
        out["deltas"][name] = [float(q.delta) for q in [block.act_quantizer] +
                               [m.act_quantizer for m in block.modules()
                                if hasattr(m, "act_quantizer") and m is not block]
                               if getattr(q, "delta", None) is not None]
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
