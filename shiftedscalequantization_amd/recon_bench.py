"""Reconstruction-iteration benchmark used by bench.py (the "recon iters/s" half of the
BASELINE metric): block_recon_fused_shiftedScale on ResNet-18 blocks, batch 32 per rank,
W2 shifted-scale (S=3 shifts [31/32, 33/32, 1]), lmda (0.01, 0.1), cached features of
1024 synthetic calibration samples per rank, gradients all-reduced over RCCL for N > 1.
"""
import time

import torch

from . import nets
from .quant import ChannelQuant, QuantModel, QuantModule
from .quant.layer_recon_fused_shiftedScale import block_recon_fused_shiftedScale

SHIFTS = [31 / 32, 33 / 32, 1.0]
# block -> (input shape per sample)
BLOCKS = {"layer1.0": (64, 56, 56), "layer2.0": (64, 56, 56), "layer3.0": (128, 28, 28),
          "layer4.0": (256, 14, 14)}


def _block(qnn, name):
    m = qnn.model if hasattr(qnn, "model") else qnn
    for part in name.split("."):
        m = m[int(part)] if part.isdigit() else getattr(m, part)
    return m


def _block_input_shape(cnn, name, dev):
    """Per-sample input shape of block `name` of the FP model (one 224x224 forward)."""
    shape = {}

    def hook(m, i, o):
        shape.setdefault("s", i[0].shape)

    h = _block(cnn, name).register_forward_hook(hook)
    with torch.no_grad():
        cnn(torch.zeros(1, 3, 224, 224, device=dev))
    h.remove()
    return tuple(shape["s"][1:])


def run_block(dev, name, n_cali=1024, iters=200, warmup=20, rank=0, bias_cal=False,
              arch="resnet18"):
    torch.manual_seed(1005 + rank)
    cnn = nets.ARCHS[arch]().eval()
    # (on the host: a device forward under cudnn.benchmark would tune every conv of the net)
    in_shape = BLOCKS[name] if arch == "resnet18" else _block_input_shape(cnn, name, "cpu")
    cnn = cnn.to(dev)
    qnn = QuantModel(cnn, {"n_bits": 2, "channel_wise": True, "scale_method": "max"},
                     {"n_bits": 4, "channel_wise": False, "scale_method": "mse", "leaf_param": True})
    qnn.to(dev).eval()
    qnn.set_first_last_layer_to_8bit()
    block = _block(qnn, name)
    for m in block.modules():
        if isinstance(m, QuantModule):
            m.weight_quantizer.channel_wise = True
            with torch.no_grad():
                m.weight_quantizer(m.org_weight)           # 'max' init on the device
            m.weight_quantizer = ChannelQuant(1.0, uaq=m.weight_quantizer, weight_tensor=m.org_weight,
                                              shiftTarget=SHIFTS, name=name)
    g = torch.Generator(device=dev).manual_seed(1005 + rank)
    inp = torch.empty((n_cali,) + in_shape, device=dev).normal_(generator=g).relu_()
    with torch.no_grad():
        block.set_quant_state(False, False)
        out = torch.cat([block(inp[i:i + 64]) for i in range(0, n_cali, 64)])
    block.set_quant_state_block(True)
    block.cached_inp_features, block.cached_out_features = [inp], [out]
    stamps = {}

    def hook(i):
        if i in (warmup, warmup + iters):
            torch.cuda.synchronize(dev)
            stamps[i] = time.perf_counter()

    import builtins
    _print = builtins.print
    builtins.print = lambda *a, **k: None       # silence the loop's init prints
    try:
        block_recon_fused_shiftedScale(block, warmup + iters, (0.01, 0.1), qnn, None, verbose=False,
                                       iter_hook=hook, bias_cal=bias_cal)
    finally:
        builtins.print = _print
    dt = stamps[warmup + iters] - stamps[warmup]
    return iters / dt


def _rate(dev, world, rank, name, iters):
    ips = run_block(dev, name, iters=iters, rank=rank)
    if world > 1:
        import torch.distributed as dist
        t = torch.tensor([1.0 / ips], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)     # slowest rank sets the pace
        ips = 1.0 / t.item()
    return round(ips, 2)


def run_recon_bench(dev, world, rank, iters=200, blocks=("layer1.0", "layer4.0")):
    """iters/s per block with MIOpen's measured solver choice (cudnn.benchmark: miopenFind
    once per shape, during the eager warm-up) and, beside it, under the reference's
    seed_all setting (cudnn.deterministic, benchmark off: MIOpen's deterministic solvers,
    K17 for the weight gradients where those are slow, kernels.WGRAD_POLICY)."""
    cudnn = torch.backends.cudnn
    saved = (cudnn.benchmark, cudnn.deterministic)
    res, res_det = {}, {}
    try:
        for b in blocks:
            cudnn.benchmark, cudnn.deterministic = True, False
            res[b] = _rate(dev, world, rank, b, iters)
            cudnn.benchmark, cudnn.deterministic = False, True
            res_det[b] = _rate(dev, world, rank, b, iters)
    finally:
        cudnn.benchmark, cudnn.deterministic = saved
    return {"metric": "block_recon_fused_shiftedScale iters/s (batch 32 per rank, W2, S=3)",
            "iters_per_s": res, "conv_solvers": "MIOpen find (cudnn.benchmark)",
            "iters_per_s_deterministic": res_det, "timed_iters": iters, "n_gpus": world,
            "samples_per_s": {k: round(v * 32 * world, 1) for k, v in res.items()}}
