"""Reconstruction-iteration benchmark used by bench.py (the "recon iters/s" half of the
BASELINE metric): block_recon_fused_shiftedScale on every ResNet-18 block (layer1.0 ...
layer4.1), batch 32 per rank, W2 shifted-scale (S=3 shifts [31/32, 33/32, 1]),
lmda (0.01, 0.1), bias_cal (gamma^z/phi^z learned, the README's --bias_cal), cached
features of 1024 synthetic calibration samples per rank, gradients all-reduced over RCCL
for N > 1.

Rates are measured under the reference's seed_all setting (cudnn.deterministic: MIOpen's
deterministic solvers, K17 for the weight gradients it is slow at) -- the headline -- and
beside it with MIOpen's measured solver choice (cudnn.benchmark).  The SURVEY §8(d) recon
roofline is priced on the loop's own launches: tools/recon_roofline.py reads a rocprofv3
kernel trace of these loops (profiles/recon_roofline.json, which bench.py reports).
"""
import time

import torch

from . import kernels as K
from . import nets
from .quant import ChannelQuant, QuantModel, QuantModule
from .quant.layer_recon_fused_shiftedScale import block_recon_fused_shiftedScale

SHIFTS = [31 / 32, 33 / 32, 1.0]
# block -> per-sample input shape (ResNet-18 at 224x224)
BLOCKS = {"layer1.0": (64, 56, 56), "layer1.1": (64, 56, 56), "layer2.0": (64, 56, 56),
          "layer2.1": (128, 28, 28), "layer3.0": (128, 28, 28), "layer3.1": (256, 14, 14),
          "layer4.0": (256, 14, 14), "layer4.1": (512, 7, 7)}


def graph_time_ms(fn, reps=20, rounds=5):
    """Device time per call of `fn`: `reps` calls captured in one HIP graph (no host
    launch cost), replayed `rounds` times, median of the per-replay averages (HIP events on
    the capturing stream)."""
    fn()
    torch.cuda.synchronize()
    graph, ws = torch.cuda.CUDAGraph(), {}
    with K.A.workspace_scope(ws):
        with torch.cuda.graph(graph):
            for _ in range(reps):
                fn()
    graph.replay()
    torch.cuda.synchronize()
    times = []
    for _ in range(rounds):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        graph.replay()
        b.record()
        torch.cuda.synchronize()
        times.append(a.elapsed_time(b) / reps)
    del graph
    return sorted(times)[len(times) // 2]


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


def _cpu_state(block, inp, tgt):
    """Host copies of what oracle/recon_cpu.FusedBlockReconCPU needs for this block."""
    convs = {}
    for n in ("conv1", "conv2", "downsample"):
        m = getattr(block, n, None)
        if m is None:
            continue
        q = m.weight_quantizer
        convs[n] = (m.org_weight.detach().cpu(), m.org_bias.detach().cpu(), q.delta.detach().cpu(),
                    q.zero_point.detach().cpu(), int(m.fwd_kwargs["stride"][0]),
                    int(m.fwd_kwargs["padding"][0]))
    return {"convs": convs, "inp": inp.detach().cpu(), "out": tgt.detach().cpu()}


def run_block(dev, name, n_cali=1024, iters=200, warmup=20, rank=0, bias_cal=True,
              arch="resnet18", cpu_sample=0):
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
    res = {}
    if cpu_sample:
        res["cpu_state"] = _cpu_state(block, inp[:cpu_sample], out[:cpu_sample])
    stamps = {}

    def hook(i):
        if i in (warmup, warmup + iters):
            torch.cuda.synchronize(dev)
            stamps[i] = time.perf_counter()

    import builtins
    from . import parallel_dp as P
    _print = builtins.print
    builtins.print = lambda *a, **k: None       # silence the loop's init prints
    P.TIMING = [] if P.world() > 1 else None
    try:
        block_recon_fused_shiftedScale(block, warmup + iters, (0.01, 0.1), qnn, None, verbose=False,
                                       iter_hook=hook, bias_cal=bias_cal)
        torch.cuda.synchronize(dev)
        if P.TIMING:
            # the gradient all-reduce of the timed iterations (one bucket per iteration)
            ev = P.TIMING[-iters:]
            res["allreduce_us"] = sum(a.elapsed_time(b) for a, b, _ in ev) / len(ev) * 1e3
            res["bucket_bytes"] = 4 * ev[-1][2]
    finally:
        builtins.print = _print
        P.TIMING = None
    res["ips"] = iters / (stamps[warmup + iters] - stamps[warmup])
    return res


def _slowest(ips, world, dev):
    if world > 1:
        import torch.distributed as dist
        t = torch.tensor([1.0 / ips], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)     # slowest rank sets the pace
        ips = 1.0 / t.item()
    return ips


def run_recon_bench(dev, world, rank, iters=200, blocks=tuple(BLOCKS), bias_cal=True,
                    cpu_sample=0):
    """iters/s of every block under cudnn.deterministic (the reference's seed_all, the
    headline) and under cudnn.benchmark, and (cpu_sample > 0) layer1.0's state for the CPU
    baseline."""
    cudnn = torch.backends.cudnn
    saved = (cudnn.benchmark, cudnn.deterministic)
    det, fast, cpu_state, coll = {}, {}, None, {}
    try:
        for b in blocks:
            cudnn.benchmark, cudnn.deterministic = False, True
            r = run_block(dev, b, iters=iters, rank=rank, bias_cal=bias_cal,
                          cpu_sample=cpu_sample if (b == blocks[0] and rank == 0) else 0)
            det[b] = round(_slowest(r["ips"], world, dev), 2)
            cpu_state = r.get("cpu_state", cpu_state)
            if "allreduce_us" in r:
                us = r["allreduce_us"]
                coll[b] = {"allreduce_us_per_iter": round(us, 2), "bucket_bytes": r["bucket_bytes"],
                           "share_of_iteration": round(us * 1e-6 * r["ips"], 4)}
            cudnn.benchmark, cudnn.deterministic = True, False
            fast[b] = round(_slowest(run_block(dev, b, iters=iters, rank=rank,
                                               bias_cal=bias_cal)["ips"], world, dev), 2)
    finally:
        cudnn.benchmark, cudnn.deterministic = saved
    # one fused iteration of every block = one "ResNet-18 recon iteration"
    model_det = 1.0 / sum(1.0 / v for v in det.values())
    model_fast = 1.0 / sum(1.0 / v for v in fast.values())
    out = {"metric": "block_recon_fused_shiftedScale iters/s (batch 32 per rank, W2, S=3, bias_cal)",
           "conv_solvers": "cudnn.deterministic (reference seed_all; headline) | cudnn.benchmark",
           "iters_per_s": det, "iters_per_s_benchmark_solvers": fast,
           "resnet18_all_blocks_iters_per_s": round(model_det, 2),
           "resnet18_all_blocks_iters_per_s_benchmark_solvers": round(model_fast, 2),
           "timed_iters": iters, "n_gpus": world,
           "samples_per_s": {k: round(v * 32 * world, 1) for k, v in det.items()}}
    if coll:
        # rank 0's view of the per-iteration gradient all-reduce (deterministic-solver loops)
        out["allreduce_per_block"] = coll
        out["allreduce_backend"] = torch.distributed.get_backend()
    if cpu_state is not None:
        out["_cpu_state"] = cpu_state
    return out
