"""Benchmark of the shifted-scale calibration hot path on MI355X (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...

`--gpus N` alone starts its own N rank processes (shiftedscalequantization_amd/launch.py, as
the reference's mp.spawn, Brecq/main_imagenet_dist.py:268-271); under an external launcher
(WORLD_SIZE set) this process is one rank.

One step (configs[1], ResNet-18 W2A4, 1024 calibration samples, synthetic data) =
  * A4 per-tensor q/dq of the block-input activation cache [1024,64,56,56] fp32
    (205.5 M elements, 822 MB >> the 256 MB Infinity Cache), delta/zp from the 'mse'
    init on the first 64 samples, and
  * W2 per-channel q/dq of every ResNet-18 conv/fc weight (11.68 M elements, 8-bit
    stem/head), as one multi-tensor table riding on the activation's launch
    (K.deferred_fq_multi): the whole step is ONE kernel launch.
value = elements processed by all ranks / max-over-ranks wall time (Gelem/s, weak
scaling: every rank owns its own calibration shard; no data-path collective).
The reconstruction iteration rate (block_recon_fused_shiftedScale, batch 32, bias_cal, every
ResNet-18 block, reference-faithful deterministic conv solvers as the headline) is reported
beside it as `recon`, with its SURVEY §8(d) roofline as `roofline_recon` (priced on the
loop's own kernel launches from a rocprofv3 trace of these loops: tools/recon_roofline.py).
"""
import argparse
import json
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

if __name__ == "__main__":
    # --gpus N > 1 without an external launcher: start N rank processes of this script now,
    # before torch (and the HIP runtime) is loaded in this parent (launch.py)
    from shiftedscalequantization_amd.launch import maybe_spawn
    maybe_spawn(os.path.abspath(__file__))

# MIOpen persists its solver choices in a per-user find-db that outlives the process: a
# test run that convolved under cudnn.deterministic would otherwise hand its (slow,
# deterministic) solvers to this bench's recon loops on the same box.  Fresh db per run.
os.environ.setdefault("MIOPEN_USER_DB_PATH", tempfile.mkdtemp(prefix="ssq_bench_miopen_"))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from shiftedscalequantization_amd import kernels as K  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
RESNET18_SHAPES = ([(64, 3, 7, 7)] + [(64, 64, 3, 3)] * 4 +
                   [(128, 64, 3, 3), (128, 128, 3, 3), (128, 64, 1, 1), (128, 128, 3, 3),
                    (128, 128, 3, 3)] +
                   [(256, 128, 3, 3), (256, 256, 3, 3), (256, 128, 1, 1), (256, 256, 3, 3),
                    (256, 256, 3, 3)] +
                   [(512, 256, 3, 3), (512, 512, 3, 3), (512, 256, 1, 1), (512, 512, 3, 3),
                    (512, 512, 3, 3)] + [(1000, 512)])


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    # 20 warm-up + >= 100 timed repetitions (30 ms of GPU time)
    p.add_argument("--steps", type=int, default=100)
    p.add_argument("--warmup", type=int, default=20)
    p.add_argument("--n-cali", type=int, default=1024)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-seconds", type=float, default=15.0)
    p.add_argument("--no-recon", action="store_true")
    p.add_argument("--recon-iters", type=int, default=200)
    p.add_argument("--no-validate", action="store_true")
    p.add_argument("--no-recon-configs", action="store_true",
                   help="skip BASELINE configs 3-5's loops (recon_configs)")
    p.add_argument("--variant", type=int, default=-1, help="streaming cache policy A/B")
    p.add_argument("--dist-backend", default="nccl",
                   help="nccl (= RCCL over xGMI, the default) or gloo (rehearsing N > 1 ranks "
                        "on fewer GPUs: ranks share devices round-robin)")
    return p.parse_args()


def setup(backend="nccl"):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    ndev = torch.cuda.device_count()
    if world > 1 and backend == "nccl" and world > ndev:
        raise SystemExit(f"bench.py: {world} ranks over RCCL need {world} GPUs, {ndev} visible "
                         f"(rehearse with --dist-backend gloo: ranks then share devices)")
    dev = torch.device("cuda", local % max(ndev, 1))
    torch.cuda.set_device(dev)
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)
    return rank, world, dev


def barrier(world):
    if world > 1:
        dist.barrier()


def max_over_ranks(v, world, dev):
    if world == 1:
        return v
    t = torch.tensor([v], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return t.item()


def make_workload(dev, rank, n_cali):
    g = torch.Generator(device=dev).manual_seed(1005 + rank)
    act = torch.empty(n_cali, 64, 56, 56, device=dev)
    act.normal_(generator=g).relu_()
    d_a, z_a, _ = K.scale_init(act[:64], 4, False, False, "mse")
    weights, dws, zws, bits = [], [], [], []
    for i, s in enumerate(RESNET18_SHAPES):
        w = torch.empty(s, device=dev).normal_(0.0, 0.02, generator=g)
        b = 8 if i in (0, len(RESNET18_SHAPES) - 1) else 2
        d, z, _ = K.scale_init(w, b, False, True, "max")
        weights.append(w)
        dws.append(d)
        zws.append(z)
        bits.append(b)
    return act, d_a, z_a, weights, dws, zws, bits


PMC_FILE = "profiles/pmc_traffic.json"


def _stamp(d):
    """Provenance of a committed measurement summary against the tree this bench runs from:
    the source hash it was measured at (shiftedscalequantization_amd.build.source_sha) and
    stale = True when the kernels changed since, or when it carries no stamp."""
    from shiftedscalequantization_amd.build import source_sha
    prov = d.get("provenance") or {}
    return {"measured_at_git": prov.get("git_sha"), "measured_at_csrc": prov.get("csrc_sha"),
            "csrc_now": source_sha(), "stale": prov.get("csrc_sha") != source_sha()}


def pmc_traffic(kernel="fq_fwd_pt"):
    """(HBM bytes per launch of `kernel`, provenance) from the committed rocprofv3 PMC passes
    (tools/session.sh TAG pmc: FETCH_SIZE and WRITE_SIZE in separate passes, read side doubled
    per the gfx950 correction), or (None, None) if they were not collected."""
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), PMC_FILE)
    try:
        with open(path) as f:
            d = json.load(f)
        return float(d[kernel]["hbm_bytes_per_launch"]), _stamp(d)
    except (OSError, KeyError, ValueError):
        return None, None


RECON_ROOFLINE_FILE = "profiles/recon_roofline.json"


def recon_roofline():
    """SURVEY §8(d) recon roofline priced on the loop's own launches: the summary that
    tools/recon_roofline.py wrote from a rocprofv3 kernel trace of this bench's recon loops
    (per block, per kernel class: time and algorithmic bytes), or None."""
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), RECON_ROOFLINE_FILE)
    try:
        with open(path) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return None
    out = {k: v for k, v in d.items() if k not in ("blocks", "provenance")}
    out["source_file"] = RECON_ROOFLINE_FILE + " (a committed trace, not this run)"
    out.update(_stamp(d))
    out["per_block_gbs"] = {b: v["achieved_gbs"] for b, v in d.get("blocks", {}).items()}
    return out


RECON_CONFIGS_ROOFLINE_FILE = "profiles/recon_configs_roofline.json"


def recon_configs_roofline():
    """Configs 3-5's ssq-set rooflines: the summary tools/recon_roofline.py --configs wrote
    from a rocprofv3 kernel trace of these loops, or None."""
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), RECON_CONFIGS_ROOFLINE_FILE)
    try:
        with open(path) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return None
    out = {k: v for k, v in d.items() if k != "provenance"}
    out["source_file"] = RECON_CONFIGS_ROOFLINE_FILE + " (a committed trace, not this run)"
    out.update(_stamp(d))
    return out


def time_events(fn, reps, dev, rounds=5):
    """Average launch time (ms) of fn over `reps` back-to-back launches, measured with HIP
    events on the current stream; the median of `rounds` such groups (after one untimed
    warm-up launch) so that a clock ramp or one slow group does not set the number."""
    fn()
    times = []
    for _ in range(rounds):
        start, end = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        start.record()
        for _ in range(reps):
            fn()
        end.record()
        torch.cuda.synchronize(dev)
        times.append(start.elapsed_time(end) / reps)
    return sorted(times)[len(times) // 2]


def host_cores():
    """The host CPU share this process may use: OMP_NUM_THREADS when the box sets it (its
    per-GPU share), else the affinity mask."""
    env = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    return env if env > 0 else len(os.sched_getaffinity(0))


def cpu_model():
    """The host CPU's model name (report it beside the CPU baseline)."""
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def _timed(fn, seconds, min_reps=2):
    fn()  # warm
    n, t0 = 0, time.perf_counter()
    while True:
        fn()
        n += 1
        el = time.perf_counter() - t0
        if el >= seconds and n >= min_reps:
            return n, el


def cpu_baseline(act_dev, d_a, z_a, seconds, recon_state=None):
    """The CPU ports on the GPU box's host cores, on bounded samples of the same workload:
    * q/dq: the plain-C oracle (oracle/c, scalar) on act[:64] (12.8 M elements), 1 thread
      and all cores (the sample split into one contiguous slice per thread; ctypes releases
      the GIL);
    * recon: oracle/recon_cpu.FusedBlockReconCPU -- the reference's fused iteration in
      PyTorch-CPU ops, pinned to the reference trajectory by tests/test_oracle.py -- on
      ResNet-18 layer1.0 (batch 32 from 64 cached samples, bias_cal), all cores."""
    import concurrent.futures as cf

    import numpy as np
    from oracle import c_oracle
    cores = host_cores()
    sample = act_dev[:64].cpu().numpy()
    d, z = d_a.cpu().numpy(), z_a.cpu().numpy()
    c_oracle.fake_quant(sample[:1], d, z, 4)  # load / warm
    n1, el1 = _timed(lambda: c_oracle.fake_quant(sample, d, z, 4), seconds / 3)
    flat = sample.reshape(-1)
    slices = np.array_split(flat, cores)
    pool = cf.ThreadPoolExecutor(max_workers=cores)

    def all_cores():
        list(pool.map(lambda x: c_oracle.fake_quant(x, d, z, 4), slices))

    nN, elN = _timed(all_cores, seconds / 3)
    pool.shutdown()
    c_port = {"value": round(nN * sample.size / elN / 1e9, 4), "unit": "Gelem/s", "cores": cores,
              "kind": "port", "value_1thread": round(n1 * sample.size / el1 / 1e9, 4),
              "sample": f"oracle/c ssqo_fake_quant (scalar C port of quant_layer.py:92-98), "
                        f"act[:64] ({sample.size} elems) x{nN} reps in {elN:.1f}s on {cores} "
                        f"threads"}
    # the reference's own CPU path -- the headline baseline: its eager torch op sequence
    # (oracle/torch_eager.py, quant_layer.py:18-22,92-98) on the same sample, all cores and
    # one thread
    import torch
    from oracle.torch_eager import uaq_fake_quant
    xs, dt, zt = torch.from_numpy(sample), torch.from_numpy(d), torch.from_numpy(z)
    prev = torch.get_num_threads()
    eager, eager_n = {}, {}
    for nt in (cores, 1):
        torch.set_num_threads(nt)
        ne, ele = _timed(lambda: uaq_fake_quant(xs, dt, zt, 4), seconds / 6)
        eager[nt] = round(ne * sample.size / ele / 1e9, 4)
        eager_n[nt] = (ne, ele)
    torch.set_num_threads(prev)
    out = {"value": eager[cores], "unit": "Gelem/s", "cores": cores,
           # a restatement (the reference's source cannot travel to the GPU box), op for op
           "kind": "port",
           "sample": f"the reference's UniformAffineQuantizer.forward op sequence "
                     f"(quant_layer.py:18-22,92-98: x/delta, round_ste, +zp, clamp, -zp, *delta) "
                     f"as torch-CPU eager ops on act[:64] ({sample.size} elems, A4 per-tensor), "
                     f"x{eager_n[cores][0]} reps in {eager_n[cores][1]:.1f}s on {cores} torch "
                     f"threads; {os.cpu_count()} host CPUs visible",
           "value_1thread": eager[1], "cpu_model": cpu_model(), "c_port": c_port}
    if recon_state is not None:
        import torch
        from oracle.recon_cpu import FusedBlockReconCPU
        torch.set_num_threads(cores)
        torch.manual_seed(1005)
        rc = FusedBlockReconCPU(recon_state["convs"], [31 / 32, 33 / 32, 1.0], 2, recon_state["inp"],
                                recon_state["out"], 625, bias_cal=True)
        nr, elr = _timed(rc.step, seconds / 3, min_reps=3)
        out["recon_iters_per_s"] = round(nr / elr, 3)
        out["recon_sample"] = (f"oracle/recon_cpu.FusedBlockReconCPU, ResNet-18 layer1.0 W2 S=3 "
                               f"bias_cal, batch 32 of 64 cached samples, {nr} iterations in "
                               f"{elr:.1f}s on {cores} torch threads")
        torch.set_num_threads(1)
        n1r, el1r = _timed(rc.step, seconds / 6, min_reps=2)
        torch.set_num_threads(cores)
        out["recon_iters_per_s_1thread"] = round(n1r / el1r, 3)
    return out


def main():
    args = parse()
    rank, world, dev = setup(args.dist_backend)
    if world > 1 and args.gpus not in (1, world):
        print(f"bench.py: --gpus {args.gpus} but the launcher started {world} ranks; "
              f"reporting {world}", file=sys.stderr)
    if args.variant >= 0:
        K.set_variant(args.variant)
    act, d_a, z_a, weights, dws, zws, bits = make_workload(dev, rank, args.n_cali)
    y_act = torch.empty_like(act)
    n_act = act.numel()
    n_w = sum(w.numel() for w in weights)
    elems_per_step = n_act + n_w

    y_w = [torch.empty_like(w) for w in weights]
    # the 21 weights' arguments checked and packed once (a launch plan, like the weights of
    # a fixed model quantised every step); every output is written in place
    w_plan = K.FqMultiPlan(weights, dws, zws, bits, out=y_w)

    def step():
        # the weights' table rides on the activation's launch: one kernel per step
        with K.deferred_fq_multi():
            w_plan()
            K.fake_quant_fwd(act, d_a, z_a, 4, out=y_act)

    # the timed region comes after the kernel probes below, so that the W warm-up steps
    # start on a GPU whose clocks have already left idle (the driver runs --steps 20
    # --warmup 5: a 6 ms region)

    # dominant kernel: the step's one launch (fq_fwd_pt_ride: the A4 activation q/dq with
    # the weights' tiles riding on it), timed with HIP events on the stream it is launched
    # on: 20 launches replayed from a HIP graph (the step's host-side argument packing for
    # 21 weights is not kernel time), median of 9 replays; beside it the activation's q/dq
    # alone (fq_fwd_pt), 20 eager back-to-back launches
    from shiftedscalequantization_amd.recon_bench import graph_time_ms
    ms_step_k = graph_time_ms(step, reps=20, rounds=9)
    ms_fq = time_events(lambda: K.fake_quant_fwd(act, d_a, z_a, 4, out=y_act), 20, dev, rounds=9)
    # the committed PMC passes were collected on the default workload (1024 samples)
    traffic, traffic_prov = pmc_traffic("fq_fwd_pt_ride") if args.n_cali == 1024 else (None, None)
    traffic_k1, _ = pmc_traffic("fq_fwd_pt") if args.n_cali == 1024 else (None, None)
    alg_bytes = 8.0 * (n_act + n_w)
    achieved = alg_bytes / (ms_step_k * 1e-3) / 1e9
    achieved_k1 = 8.0 * n_act / (ms_fq * 1e-3) / 1e9
    # stream-copy ceiling of this box: the best of the copy geometries the q/dq kernel
    # is tuned over (1 workgroup/CU x unroll 4 / 8), same tensor, same bytes
    copy_gbs, default_variant = 0.0, K.set_variant(0)
    for v in (1 | (256 << 8), 1 | (3 << 4) | (256 << 8)):
        K.set_variant(v)
        ms_copy = time_events(lambda: K.stream_copy(act, y_act), 20, dev)
        copy_gbs = max(copy_gbs, 8.0 * n_act / (ms_copy * 1e-3) / 1e9)
    K.set_variant(default_variant)
    # the HBM's read and write paths priced separately on the same bytes: K1 moves 4 B in
    # and 4 B out per element, so its ceiling is the 1:1 harmonic mix of the two rates
    sink = torch.empty(4, device=dev)
    rd_gbs = 4.0 * n_act / (time_events(lambda: K.stream_read(act, sink), 20, dev) * 1e-3) / 1e9
    wr_gbs = 4.0 * n_act / (time_events(lambda: K.stream_write(y_act), 20, dev) * 1e-3) / 1e9
    mix_gbs = 2.0 / (1.0 / rd_gbs + 1.0 / wr_gbs)
    # all 21 weights in one launch: device time from a HIP-graph replay (no host launch
    # cost), beside the eager host-launch rate of the same call
    ms_w = graph_time_ms(lambda: K.fake_quant_multi(weights, dws, zws, bits))
    ms_w_launch = time_events(lambda: K.fake_quant_multi(weights, dws, zws, bits), 20, dev)
    # W2 per-channel q/dq of the large synthetic weight of BASELINE.md §2 ([8192,2048,3,3],
    # per-output-channel delta/zp staged in LDS): the per-channel kernel's roofline line
    big = torch.empty(8192, 2048, 3, 3, device=dev).normal_(0.0, 0.02)
    d_big, z_big, _ = K.scale_init(big, 2, False, True, "max")
    y_big = torch.empty_like(big)
    ms_pc = time_events(lambda: K.fake_quant_fwd(big, d_big, z_big, 2, out=y_big), 10, dev)
    pc_gbs = 8.0 * big.numel() / (ms_pc * 1e-3) / 1e9
    del big, y_big

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    barrier(world)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize(dev)
    barrier(world)
    elapsed = max_over_ranks(time.perf_counter() - t0, world, dev)
    value = world * elems_per_step * args.steps / elapsed / 1e9

    recon = None
    recon_state = None
    recon_configs = None
    if not args.no_recon:
        from shiftedscalequantization_amd.recon_bench import run_recon_bench
        want_cpu = world == 1 and rank == 0 and not args.no_cpu_baseline
        recon = run_recon_bench(dev, world, rank, iters=args.recon_iters,
                                cpu_sample=64 if want_cpu else 0)
        recon_state = recon.pop("_cpu_state", None)
        if not args.no_recon_configs:
            from shiftedscalequantization_amd.recon_bench import run_recon_configs
            recon_configs = run_recon_configs(dev, world, rank, iters=args.recon_iters)

    validation = None
    if not args.no_validate:
        from shiftedscalequantization_amd.validate_bench import run_validate_bench
        validation = run_validate_bench(dev, world, rank)
        el = max_over_ranks(validation.pop("_elapsed_s"), world, dev)
        validation["images_per_s"] = round(world * validation["_images"] / el, 1)
        validation.pop("_images")

    out = {
        "metric": "Gelem/s shifted-scale q/dq + recon iters/s, ResNet-18 W2A4; top-1 vs ref",
        "value": round(value, 3),
        "unit": "Gelem/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic (ReLU(N(0,1)) activation cache, N(0,0.02^2) ResNet-18-shaped weights)",
        "config": {"workload": "resnet18 W2A4 bias_cal+bias_ch_quant, 1024 calib samples: A4 "
                               "per-tensor q/dq of act [1024,64,56,56] + W2 per-channel q/dq of "
                               "all 21 conv/fc weights (8-bit stem/head)",
                   "elems_per_step_per_rank": elems_per_step, "parallelism": f"dp{world}"},
        # how the ranks came to be and what the process group saw (n_gpus is the latter)
        "launch": {"launcher": os.environ.get("SSQ_LAUNCHER",
                                              "external" if "WORLD_SIZE" in os.environ else "none"),
                   "world_size_backend": dist.get_world_size() if world > 1 else 1,
                   "allreduce_backend": dist.get_backend() if world > 1 else None,
                   "devices_visible": torch.cuda.device_count()},
        "roofline": {"bound": "hbm",
                     "kernel": "fq_fwd_pt_ride (ssq_fq_fwd per-tensor A4 with the 21 weights' "
                               "ssq_fq_fwd_multi tiles riding on the launch: the whole step)",
                     "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                     "traffic_source": (PMC_FILE + " (committed PMC passes, not this run)")
                                       if traffic is not None else None,
                     "traffic_provenance": traffic_prov,
                     "kernel_ms": round(ms_step_k, 4), "alg_bytes_per_launch": int(alg_bytes),
                     "k1_alone": {"kernel": "fq_fwd_pt (A4 activation only)",
                                  "kernel_ms": round(ms_fq, 4),
                                  "alg_bytes_per_launch": int(8.0 * n_act),
                                  "achieved": round(achieved_k1, 1),
                                  "frac": round(achieved_k1 / HBM_PEAK_GBS, 4),
                                  "traffic": traffic_k1},
                     "stream_copy_gbs": round(copy_gbs, 1),
                     "frac_of_stream_copy": round(achieved / copy_gbs, 4),
                     "read_only_gbs": round(rd_gbs, 1), "write_only_gbs": round(wr_gbs, 1),
                     "mixed_rw_ceiling_gbs": round(mix_gbs, 1),
                     "frac_of_mixed_rw_ceiling": round(achieved / mix_gbs, 4)},
        "weights_multi_ms": round(ms_w, 4),
        "weights_multi_ms_source": "HIP-graph replay of the one-launch W2/W8 q/dq of all 21 "
                                   "weights (11.68 M elems): kernel time",
        "weights_multi_launch_ms": round(ms_w_launch, 4),
        "roofline_per_channel": {"kernel": "fq_fwd_multi_kernel (ssq_fq_fwd per-channel, 1 segment)",
                                 "workload": "W2 per-channel q/dq of [8192,2048,3,3] (151 M elems)",
                                 "achieved": round(pc_gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                 "frac": round(pc_gbs / HBM_PEAK_GBS, 4), "kernel_ms": round(ms_pc, 4)},
    }
    if recon is not None:
        rr = recon_roofline()
        if rr is not None:
            out["roofline_recon"] = rr
        out["recon"] = recon
    if recon_configs is not None:
        rc = recon_configs_roofline()
        if rc is not None:
            keep = ("wall_us_per_iteration", "ssq_set_us", "ssq_set_bytes", "achieved", "peak",
                    "unit", "frac", "conv_side_ssq_kernels_us", "library_convs_gemms_other_us")
            for k, v in recon_configs.items():
                # one roofline per loop: config3's two phases, the fused loop of configs 4 / 5
                loops = {kk: vv for kk, vv in rc.get("configs", {}).items()
                         if kk == k or kk.startswith(k + "_")}
                if loops:
                    v["roofline"] = {kk[len(k) + 1:] or "fused_loop":
                                     {f: vv[f] for f in keep if f in vv} for kk, vv in loops.items()}
            recon_configs["roofline_source"] = {kk: vv for kk, vv in rc.items() if kk != "configs"}
        out["recon_configs"] = recon_configs
    if validation is not None:
        out["validation"] = validation
    if world == 1 and rank == 0 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(act, d_a, z_a, args.cpu_seconds, recon_state)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
