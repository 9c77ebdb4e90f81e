"""W2A4 fake-quant validation inference benchmark used by bench.py.

The reference validates its calibrated network with `common.validate_model`
(common.py:152-221): a plain forward of the QuantModel with weights and activations
fake-quantized.  Here that forward is MIOpen's conv + the fused K13 epilogue (bias,
residual, ReLU and the A4 activation q/dq in one pass, `ssq_bias_act_fq`) + the W2/W8
per-channel weight q/dq (K1) of every layer, under torch.no_grad; as in validate_model, each
layer's W_hat is quantized once per validation pass (quant_layer.frozen_weight_cache).

Workload: ResNet-18 (random init), weights UAQ 'mse' per channel W2 (8-bit stem/head), act
UAQ 'mse' A4 initialised on 32 synthetic images, network output unquantized
(disable_network_output_quantization), 224x224 synthetic images, batch 128 per rank.
Reported: images/s per rank, and all ranks' images over the slowest rank's time (each
rank validates its own shard; the (correct, total) all-reduce is one 16-byte collective
per validation pass, outside the per-batch loop, so it is not timed).
"""
import time

import torch

from .drivers import build_qnn
from .quant.quant_layer import frozen_weight_cache


def run_validate_bench(dev, world, rank, batch=128, iters=20, warmup=3):
    torch.manual_seed(1005 + rank)
    qnn = build_qnn("resnet18", 2, 4, device=dev)
    qnn.set_quant_state(True, True)
    with torch.no_grad():
        qnn(torch.randn(32, 3, 224, 224, device=dev))
    qnn.disable_network_output_quantization()
    imgs = torch.randn(batch, 3, 224, 224, device=dev)
    with torch.no_grad():
        for _ in range(warmup):
            qnn(imgs)
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        # as validate_model: one pass = one frozen-weight cache, its first batch (inside the
        # timed region) quantizes every weight
        with frozen_weight_cache():
            for _ in range(iters):
                qnn(imgs)
        torch.cuda.synchronize(dev)
        el = time.perf_counter() - t0
    per_rank = batch * iters / el
    return {"metric": "W2A4 fake-quant validation images/s (cli.validate_model forward)",
            "model": "resnet18 W2A4 (8-bit stem/head), 224x224, batch %d per rank" % batch,
            "images_per_s_per_rank": round(per_rank, 1),
            "ms_per_batch": round(el / iters * 1e3, 3), "n_gpus": world,
            "_elapsed_s": el, "_images": batch * iters}
