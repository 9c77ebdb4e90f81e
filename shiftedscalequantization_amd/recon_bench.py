"""Reconstruction-iteration benchmark used by bench.py (the "recon iters/s" half of the
BASELINE metric): block_recon_fused_shiftedScale on every ResNet-18 block (layer1.0 ...
layer4.1), batch 32 per rank, W2 shifted-scale (S=3 shifts [31/32, 33/32, 1]),
lmda (0.01, 0.1), bias_cal (gamma^z/phi^z learned, the README's --bias_cal), cached
features of 1024 synthetic calibration samples per rank, gradients all-reduced over RCCL
for N > 1.

Rates are measured under the reference's seed_all setting (cudnn.deterministic: MIOpen's
deterministic solvers, K17 for the weight gradients it is slow at) -- the headline -- and
beside it with MIOpen's measured solver choice (cudnn.benchmark).  For each block the
ssq kernels of one iteration are also timed on their own (HIP graph of the same launches
at the block's real shapes) for the SURVEY §8(d) recon roofline:
    bytes = 24 * N_W (adaShift fwd 12 + bwd 12) + 12 * N_out (loss: pred, target in,
            gradient out) + 8 * N_in (gather: batch rows in and out)
    achieved = bytes / (adaShift fwd + bwd + loss + gather kernel time).
"""
import time

import torch

from . import kernels as K
from . import nets
from .quant import ChannelQuant, QuantModel, QuantModule
from .quant._engine import stash_block_weights
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


def _ssq_kernel_times(block, inp, tgt, bs=32):
    """The recon iteration's ssq kernels of this block, timed on their own (training
    state: soft targets, soft rounding, regulariser on)."""
    qs = [m.weight_quantizer for m in block.modules() if isinstance(m, QuantModule)]
    dev = inp.device
    regp = torch.tensor([0.1, 5.0], device=dev)
    for q in qs:
        q.hard_round = q.hard_targets = False
        q.opt_mode = 'adaShift'
        q.beta.requires_grad_(False)            # as inside the loop: beta is not learned
        q._fused_reg = (0.0, 0.0, torch.zeros(q.alpha.numel() // q.alpha.shape[-1], device=dev), regp)
    n_w = sum(q._src.numel() for q in qs)
    t_fwd = graph_time_ms(lambda: stash_block_weights(qs))
    for q in qs:
        q._stash = None
    entries = [(q._prepared(), q._src_delta, q.zero_point, q.n_bits, q.sym) for q in qs]
    assert all(e[0] is not None for e in entries), "prepared adaShift state unavailable"
    alphas = [q.alpha for q in qs]
    gys = [torch.randn_like(q._src) for q in qs]
    reg = (0.0, 0.0, [q._fused_reg[2] for q in qs], regp)

    def fwd_bwd():
        for a in alphas:
            a.grad = None
        ys = K.adashift_prepared_multi(alphas, entries, False, reg=reg)
        torch.autograd.backward(list(ys), gys)

    t_fb = graph_time_ms(fwd_bwd)
    for a in alphas:
        a.grad = None
    for q in qs:
        q._fused_reg = None
    idx = torch.randperm(inp.shape[0], device=dev)[:bs]
    buf = torch.empty((bs,) + tuple(inp.shape[1:]), device=dev)
    t_gather = graph_time_ms(lambda: K.gather_rows2(inp, idx, out0=buf))
    with torch.no_grad():
        pred = block(inp[:bs]).contiguous()
    t_loss = graph_time_ms(lambda: K.lp_loss_and_grad(pred, K.Rows(tgt, idx), 2.0, relu_mask=True))
    n_out, n_in = pred.numel(), buf.numel()
    times = {"adashift_fwd_us": t_fwd * 1e3, "adashift_bwd_us": (t_fb - t_fwd) * 1e3,
             "loss_us": t_loss * 1e3, "gather_us": t_gather * 1e3}
    bytes_ = 24 * n_w + 12 * n_out + 8 * n_in
    tot = sum(times.values())
    return {**{k: round(v, 2) for k, v in times.items()}, "weights": n_w, "out_elems": n_out,
            "in_elems": n_in, "bytes": bytes_, "ssq_us": round(tot, 2),
            "achieved_gbs": round(bytes_ / (tot * 1e-6) / 1e9, 1)}


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
              arch="resnet18", kernels=False, cpu_sample=0):
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
    _print = builtins.print
    builtins.print = lambda *a, **k: None       # silence the loop's init prints
    try:
        block_recon_fused_shiftedScale(block, warmup + iters, (0.01, 0.1), qnn, None, verbose=False,
                                       iter_hook=hook, bias_cal=bias_cal)
    finally:
        builtins.print = _print
    res["ips"] = iters / (stamps[warmup + iters] - stamps[warmup])
    if kernels:
        res["ssq"] = _ssq_kernel_times(block, inp, out)
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
    headline) and under cudnn.benchmark, the §8(d) recon roofline from the per-block ssq
    kernel times, and (cpu_sample > 0) layer1.0's state for the CPU baseline."""
    cudnn = torch.backends.cudnn
    saved = (cudnn.benchmark, cudnn.deterministic)
    det, fast, ssq, cpu_state = {}, {}, {}, None
    try:
        for b in blocks:
            cudnn.benchmark, cudnn.deterministic = False, True
            r = run_block(dev, b, iters=iters, rank=rank, bias_cal=bias_cal, kernels=True,
                          cpu_sample=cpu_sample if (b == blocks[0] and rank == 0) else 0)
            det[b] = round(_slowest(r["ips"], world, dev), 2)
            ssq[b] = r["ssq"]
            cpu_state = r.get("cpu_state", cpu_state)
            cudnn.benchmark, cudnn.deterministic = True, False
            fast[b] = round(_slowest(run_block(dev, b, iters=iters, rank=rank,
                                               bias_cal=bias_cal)["ips"], world, dev), 2)
    finally:
        cudnn.benchmark, cudnn.deterministic = saved
    # one fused iteration of every block = one "ResNet-18 recon iteration"
    model_det = 1.0 / sum(1.0 / v for v in det.values())
    model_fast = 1.0 / sum(1.0 / v for v in fast.values())
    tot_bytes = sum(v["bytes"] for v in ssq.values())
    tot_us = sum(v["ssq_us"] for v in ssq.values())
    out = {"metric": "block_recon_fused_shiftedScale iters/s (batch 32 per rank, W2, S=3, bias_cal)",
           "conv_solvers": "cudnn.deterministic (reference seed_all; headline) | cudnn.benchmark",
           "iters_per_s": det, "iters_per_s_benchmark_solvers": fast,
           "resnet18_all_blocks_iters_per_s": round(model_det, 2),
           "resnet18_all_blocks_iters_per_s_benchmark_solvers": round(model_fast, 2),
           "timed_iters": iters, "n_gpus": world,
           "samples_per_s": {k: round(v * 32 * world, 1) for k, v in det.items()},
           "ssq_kernels_per_block": ssq,
           "roofline_recon": {"bound": "hbm", "kernels": "adaShift fwd (K5p) + bwd (K6p) + lp_loss "
                                                         "(K11) + gather (K14), all 8 blocks",
                              "bytes_per_iteration": tot_bytes, "ssq_us_per_iteration": round(tot_us, 2),
                              "achieved": round(tot_bytes / (tot_us * 1e-6) / 1e9, 1), "peak": 8000.0,
                              "unit": "GB/s",
                              "frac": round(tot_bytes / (tot_us * 1e-6) / 1e9 / 8000.0, 4)}}
    if cpu_state is not None:
        out["_cpu_state"] = cpu_state
    return out
