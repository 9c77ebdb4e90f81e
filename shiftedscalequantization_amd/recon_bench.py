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


# tools/recon_configs_trace.py: MARK[0] = callable(n) launches a marker kernel at the start
# (n None) and the end (n = timed iterations) of every timed region, for a kernel trace
MARK = [None]
# tools/recon_configs_trace.py: ITER_NOTE[0] = callable(i) is told the index of every
# iteration the loop issues on the host (eager, captured, or a chunk's first)
ITER_NOTE = [None]


def _mark(n):
    if MARK[0] is not None:
        MARK[0](n)


def _note(i):
    if ITER_NOTE[0] is not None:
        ITER_NOTE[0](i)


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
        _note(i)
        if i in (warmup, warmup + iters):
            torch.cuda.synchronize(dev)
            stamps[i] = time.perf_counter()
            _mark(i - warmup if i == warmup + iters else None)

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


def run_brecq_block(dev, arch, name, n_cali=1024, iters=200, warmup=20, rank=0, act=True):
    """BRECQ block_reconstruction (quant/block_recon.py:10-116) on one block of `arch` as
    Brecq/main_imagenet.py's recon_model runs it for config 3: the AdaRound weight phase (asym,
    weight 0.01, b (20, 2), warm-up 0.2), then after the act-delta init the act phase (lr 4e-4,
    p 2.4); batch 32 drawn from the block features of n_cali synthetic 224x224 images
    (captured by the loop itself, save_inp_oup_data).  The iterations are timed on the
    production loop -- chunked graph replays -- through block_recon.TIMING_HOOK, from the first
    replay that starts at or after `warmup`."""
    from .quant import block_recon as BRm
    from .quant import block_reconstruction
    torch.manual_seed(1005 + rank)
    cnn = nets.ARCHS[arch]().eval().to(dev)
    qnn = QuantModel(cnn, {"n_bits": 2, "channel_wise": True, "scale_method": "max"},
                     {"n_bits": 4, "channel_wise": False, "scale_method": "mse", "leaf_param": True})
    qnn.to(dev).eval()
    qnn.set_first_last_layer_to_8bit()
    g = torch.Generator(device=dev).manual_seed(1005 + rank)
    cali = torch.empty(n_cali, 3, 224, 224, device=dev).normal_(generator=g)
    qnn.set_quant_state(True, False)
    with torch.no_grad():
        qnn(cali[:32])                      # every weight quantizer's 'max' init
    block = _block(qnn, name)
    total = warmup + iters
    res = {}

    def timed(phase, **kw):
        st = {}

        def hook(i):
            _note(i)
            if "t0" not in st and i >= warmup:
                torch.cuda.synchronize(dev)
                st["t0"], st["i0"] = time.perf_counter(), i
                _mark(None)
            elif i == total and "t0" in st:
                torch.cuda.synchronize(dev)
                st["t1"] = time.perf_counter()
                _mark(total - st["i0"])

        BRm.TIMING_HOOK = hook
        try:
            block_reconstruction(qnn, block, cali, batch_size=32, iters=total, **kw)
        finally:
            BRm.TIMING_HOOK = None
        res[phase] = (total - st["i0"]) / (st["t1"] - st["t0"])

    timed("weight", weight=0.01, asym=True, b_range=(20, 2), warmup=0.2, act_quant=False,
          opt_mode="mse")
    if act:
        qnn.set_quant_state(True, True)
        with torch.no_grad():
            qnn(cali[:64])                  # act-delta init (Brecq/main_imagenet.py:231-236)
        from .parallel_dp import world
        if world() > 1:
            # each rank initialised on its own shard: all-average, as main_imagenet.py does
            # (Brecq/main_imagenet_dist.py:210-211)
            qnn.synchorize_activation_statistics()
        qnn.disable_network_output_quantization()
        timed("act", act_quant=True, opt_mode="mse", lr=4e-4, p=2.4)
    del qnn, cnn, cali
    torch.cuda.empty_cache()
    return res


# BASELINE configs 3-5 beside ResNet-18's blocks: (config, arch, block, loop).  Config 3 runs
# BRECQ (Brecq/main_imagenet.py's recon_model); configs 4 and 5 run the --bias_ch_quant flow's
# fused shifted-scale loop with bias_cal, on the block the real-shape parity cases pin
# (tests/golden/realshape.py: mbv2_960, rgx_g9).
RECON_CONFIGS = (("3", "resnet50", "layer1.0", "brecq"),
                 ("4", "mobilenetv2", "features.16", "fused"),
                 ("5", "regnetx_3200m", "s3.b1", "fused"))


def run_recon_configs(dev, world, rank, iters=200, configs=RECON_CONFIGS):
    """iters/s of BASELINE configs 3-5's reconstruction loops under cudnn.deterministic (the
    reference's seed_all), one block each, batch 32 per rank."""
    cudnn = torch.backends.cudnn
    saved = (cudnn.benchmark, cudnn.deterministic)
    out = {}
    import builtins
    _print = builtins.print
    try:
        cudnn.benchmark, cudnn.deterministic = False, True
        for cfg, arch, name, loop in configs:
            t0 = time.perf_counter()
            builtins.print = lambda *a, **k: None     # silence the loops' init prints
            try:
                if loop == "brecq":
                    r = run_brecq_block(dev, arch, name, iters=iters, rank=rank)
                    ips = {"weight_phase": round(_slowest(r["weight"], world, dev), 2),
                           "act_phase": round(_slowest(r["act"], world, dev), 2)}
                    what = ("BRECQ block_reconstruction: AdaRound weight phase, then the act "
                            "phase (p 2.4)")
                else:
                    r = run_block(dev, name, iters=iters, rank=rank, arch=arch)
                    ips = {"fused_loop": round(_slowest(r["ips"], world, dev), 2)}
                    what = "block_recon_fused_shiftedScale, W2 S=3, bias_cal"
            finally:
                builtins.print = _print
            out[f"config{cfg}"] = {"arch": arch, "block": name, "loop": what,
                                   "iters_per_s": ips, "batch_per_rank": 32, "n_gpus": world,
                                   "timed_iters": iters,
                                   "setup_and_run_s": round(time.perf_counter() - t0, 1)}
    finally:
        cudnn.benchmark, cudnn.deterministic = saved
    return out


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
