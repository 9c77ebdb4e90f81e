"""CPU-side checks: the C ABI library loads and exports every declared symbol, the
host-side schedules / argument handling mirror the reference, the product path refuses
CPU tensors (no silent fallback), and the data-parallel bucket all-reduce (gloo, 2 ranks)."""
import os
import re
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    src = open(os.path.join(ROOT, "include", "ssq.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(ssq_[a-z0-9_]+)\s*\(", src)))


def test_header_declares_abi():
    syms = declared_symbols()
    for s in ("ssq_fq_fwd", "ssq_fq_bwd", "ssq_scale_init", "ssq_adashift_fwd", "ssq_adashift_bwd",
              "ssq_shift_init", "ssq_lp_loss", "ssq_gather_rows2", "ssq_inpscale_search"):
        assert s in syms


def test_library_exports_every_declared_symbol():
    from shiftedscalequantization_amd import _capi
    lib = _capi.load()
    missing = [s for s in declared_symbols() if not hasattr(lib, s)]
    assert not missing, missing
    # every declared symbol has a ctypes signature, and vice versa
    assert set(declared_symbols()) == set(_capi.SIGNATURES)
    assert lib.ssq_version() == 1
    assert lib.ssq_fq_bwd_workspace_size(10, 1, 1) > 0


def test_abi_argument_errors_without_gpu():
    """Argument validation happens on the host before any launch."""
    from shiftedscalequantization_amd import _capi
    lib = _capi.load()
    rc = lib.ssq_fq_fwd(None, None, None, None, None, 16, 1, 1, 1.0, 0, 3, None)
    assert rc == -1
    assert b"null" in lib.ssq_last_error()
    rc = lib.ssq_fq_fwd(None, None, None, None, None, 16, 1, 1, 1.0, 3, 3, None)
    assert rc == -1 and b"qmin" in lib.ssq_last_error()


def test_product_path_refuses_cpu_tensors():
    from shiftedscalequantization_amd import kernels as K
    from shiftedscalequantization_amd._capi import SSQError
    x = torch.randn(4, 4)
    with pytest.raises(SSQError):
        K.fake_quant_fwd(x, torch.tensor(0.1), torch.tensor(0.0), 4)


def test_schedules_match_reference(golden):
    from shiftedscalequantization_amd.quant.block_recon import LinearTempDecay
    from shiftedscalequantization_amd.quant.layer_recon_fused_shiftedScale import FusedLinearTempDecayShift
    from shiftedscalequantization_amd.quant.layer_recon_shiftedScale import LinearTempDecayShift
    g = golden("loss")
    f = FusedLinearTempDecayShift(100, 0.2, 20, 2)
    fs = FusedLinearTempDecayShift(100 * 3 / 4, 0.2, 20, 2)
    lin = LinearTempDecay(100, 0.2, 20, 2)
    lsh = LinearTempDecayShift(100, 0.2, 20, 2)
    for t in g["sched_t"]:
        t = int(t)
        assert f(t) == g["sched_fused"][t]
        assert fs(t) == g["sched_fused_shift"][t]
        assert lin(t) == g["sched_lin"][t]
        assert lsh(t) == g["sched_lsh"][t]


@pytest.mark.parametrize("lr,T", [(4e-5, 5000), (4e-4, 20000), (1e-3, 1), (4e-5, 7), (3e-3, 100)])
def test_cosine_lr_matches_torch_scheduler(lr, T):
    """The act phase's lr sequence (_engine.CosineLR) is the reference's
    CosineAnnealingLR(T_max=iters, eta_min=0.) stepped once per iteration
    (Brecq/quant/block_recon.py:56-58), equal as doubles at every step (a few past T_max
    too: the scheduler's restart branch)."""
    from shiftedscalequantization_amd.quant._engine import CosineLR
    opt = torch.optim.Adam([torch.zeros(1, requires_grad=True)], lr=lr)
    sch = torch.optim.lr_scheduler.CosineAnnealingLR(opt, T_max=T, eta_min=0.)
    mine = CosineLR(lr, T, 0.)
    for k in range(T + 3):
        opt.step()
        sch.step()
        assert mine.step() == opt.param_groups[0]["lr"], k


def test_quant_model_structure_resnet18():
    """QuantModel wraps the 21 conv/fc layers, 8 BasicBlocks, sets 8-bit stem/head and
    path names exactly as the reference (quant_model.py:15-69)."""
    from shiftedscalequantization_amd import nets
    from shiftedscalequantization_amd.quant import QuantBasicBlock, QuantModel, QuantModule
    torch.manual_seed(0)
    qnn = QuantModel(nets.resnet18(), {"n_bits": 2, "channel_wise": True, "scale_method": "max"},
                     {"n_bits": 4, "channel_wise": False, "scale_method": "mse", "leaf_param": True})
    qms = [m for m in qnn.modules() if isinstance(m, QuantModule)]
    assert len(qms) == 21
    assert sum(m.weight.numel() for m in qms) == 11678912
    assert len([m for m in qnn.modules() if isinstance(m, QuantBasicBlock)]) == 8
    qnn.set_first_last_layer_to_8bit()
    assert qms[0].weight_quantizer.n_bits == 8 and qms[-1].weight_quantizer.n_bits == 8
    assert qms[0].ignore_reconstruction
    assert qnn.model.layer2[0].pathName == ".layer2.0"
    assert qnn.model.layer2[0].downsample.pathName == ".layer2.0.downsample"


@pytest.mark.parametrize("arch,nq,nw", [("resnet50", 54, 25502912), ("mobilenetv2", 53, 3469760),
                                        ("regnetx_3200m", 81, 15232992)])
def test_quant_model_other_archs(arch, nq, nw):
    """The reference crashes here (setPathName missing on non-basic blocks).  Layer and
    weight counts are SURVEY §8(a)'s (RegNetX-3200M: 81 layers, 15.2 M weights)."""
    from shiftedscalequantization_amd import nets
    from shiftedscalequantization_amd.quant import QuantModel, QuantModule, BaseQuantBlock
    qnn = QuantModel(nets.ARCHS[arch](), {"n_bits": 2, "channel_wise": True, "scale_method": "max"},
                     {"n_bits": 4, "channel_wise": False, "scale_method": "mse", "leaf_param": True})
    qms = [m for m in qnn.modules() if isinstance(m, QuantModule)]
    assert len(qms) == nq
    assert sum(m.weight.numel() for m in qms) == nw
    assert all(b.pathName for b in qnn.modules() if isinstance(b, BaseQuantBlock))


def test_regnetx_design_space():
    """RegNetX stage widths / depths / groups from the design-space generator: the
    3200M model has 25 grouped 3x3 convs with g in {2, 4, 9, 21}."""
    import torch.nn as nn
    from shiftedscalequantization_amd import nets
    assert nets.regnet_stages(*nets.REGNETX["regnetx_3200m"]) == ([96, 192, 432, 1008], [2, 6, 15, 2],
                                                                   [48, 48, 48, 48])
    assert nets.regnet_stages(*nets.REGNETX["regnetx_600m"]) == ([48, 96, 240, 528], [1, 3, 5, 7],
                                                                  [24, 24, 24, 24])
    m = nets.ARCHS["regnetx_3200m"]()
    groups = [c.groups for c in m.modules() if isinstance(c, nn.Conv2d) and c.groups > 1]
    assert len(groups) == 25 and set(groups) == {2, 4, 9, 21}


def test_driver_flag_parsing():
    from shiftedscalequantization_amd.cli import parse_args
    a = parse_args(["--arch", "resnet18", "--n_bits_w", "2", "--n_bits_a", "4", "--bias_cal=True",
                    "--bias_ch_quant=True", "--weight=1.0", "--device_gpu=0"])
    assert a.bias_cal and a.bias_ch_quant and a.weight == 1.0 and a.n_bits_w == 2
    # the reference's argparse type=bool quirk: any non-empty string is True
    b = parse_args(["--bias_cal=False"])
    assert b.bias_cal is True


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _dp_worker(rank, world, port, out):
    import torch.distributed as dist
    from shiftedscalequantization_amd.parallel_dp import GradBucket, shard_rows
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    a = torch.nn.Parameter(torch.zeros(3, 4))
    b = torch.nn.Parameter(torch.zeros(5))
    a.grad = torch.full((3, 4), float(rank + 1))
    b.grad = torch.arange(5, dtype=torch.float32) * (rank + 1)
    GradBucket([a, b], average=False).allreduce_()
    c = torch.nn.Parameter(torch.zeros(2))
    c.grad = torch.full((2,), float(rank))
    GradBucket([c], average=True).allreduce_()
    out[rank] = (a.grad.clone(), b.grad.clone(), c.grad.clone(), shard_rows(1024))
    dist.destroy_process_group()


def test_grad_bucket_allreduce_gloo():
    world = 2
    port = _free_port()
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_dp_worker, args=(world, port, out), nprocs=world, join=True)
    for r in range(world):
        a, b, c, sh = out[r]
        assert torch.equal(a, torch.full((3, 4), 3.0))          # sum of 1 and 2
        assert torch.equal(b, torch.arange(5, dtype=torch.float32) * 3)
        assert torch.equal(c, torch.full((2,), 0.5))            # average of 0 and 1
    assert out[0][3] == (0, 512) and out[1][3] == (512, 1024)


def _replicated_worker(rank, world, port, out):
    import torch.distributed as dist
    from shiftedscalequantization_amd.parallel_dp import replicated
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    torch.manual_seed(3)
    m = torch.nn.Sequential(torch.nn.Conv2d(3, 4, 3), torch.nn.BatchNorm2d(4))
    same = replicated(m)
    with torch.no_grad():                    # one ulp on one rank, one element
        if rank == 1:
            w = m[0].weight.view(-1)
            w[5] = torch.nextafter(w[5], torch.tensor(1e9))
    out[rank] = (same, replicated(m))
    dist.destroy_process_group()


def test_replicated_check_gloo():
    """parallel_dp.replicated: identical modules on both ranks -> True; a one-ulp
    difference in one element on one rank -> False on every rank."""
    world = 2
    port = _free_port()
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_replicated_worker, args=(world, port, out), nprocs=world, join=True)
    assert out[0] == (True, False) and out[1] == (True, False)


def test_dwconv_support_query_covers_both_stages():
    """K18 accepts a depthwise shape only when the forward AND the input-gradient LDS
    stages fit (weight rows + padded planes / margined dy planes): 178x178 3x3 fits the
    forward plane alone but not the backward's, so it goes to MIOpen (host-only query)."""
    from shiftedscalequantization_amd import _capi as A
    assert A.query("ssq_dwconv_supported", 2, 32, 112, 112, 3, 3, 1, 1) == 1
    assert A.query("ssq_dwconv_supported", 2, 32, 56, 56, 5, 5, 2, 2) == 1
    assert A.query("ssq_dwconv_supported", 2, 32, 178, 178, 3, 3, 1, 1) == 0
    assert A.query("ssq_dwconv_supported", 2, 32, 180, 180, 3, 3, 1, 1) == 0


# ---- self-launch (--gpus N without an external launcher; launch.py) --------------------

def _dryrun(script, args):
    """Run an entry point with --gpus 2 and no launcher in the environment; the ranks stop
    before importing torch (SSQ_LAUNCH_DRYRUN) and print their rendezvous environment."""
    import json
    import subprocess
    import sys
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env["SSQ_LAUNCH_DRYRUN"] = "1"
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, os.path.join(root, script)] + args, env=env,
                       capture_output=True, text=True, timeout=120, cwd=root)
    assert r.returncode == 0, r.stderr
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    parent = [x["launcher_parent"] for x in lines if "launcher_parent" in x]
    ranks = sorted((x["rank_env"] for x in lines if "rank_env" in x), key=lambda e: e["RANK"])
    return parent, ranks


@pytest.mark.parametrize("script,args", [
    ("bench.py", ["--gpus", "2", "--dist-backend", "gloo", "--steps", "2", "--warmup", "1"]),
    ("main_imagenet.py", ["--gpus", "2", "--dist_backend", "gloo", "--arch", "resnet18"])])
def test_entry_points_spawn_ranks_before_touching_gpu(script, args):
    """`--gpus 2` alone starts two rank processes with torch.distributed.run's environment
    (the reference's mp.spawn, Brecq/main_imagenet_dist.py:268-271), from a parent that has
    not imported torch nor mapped the HIP runtime."""
    parent, ranks = _dryrun(script, args)
    assert parent == [{"torch_imported": False, "cuda_initialized": False,
                       "hip_runtime_mapped": False, "libssq_loaded": False}]
    assert [e["RANK"] for e in ranks] == ["0", "1"]
    assert [e["LOCAL_RANK"] for e in ranks] == ["0", "1"]
    assert all(e["WORLD_SIZE"] == "2" and e["MASTER_ADDR"] == "127.0.0.1" for e in ranks)
    assert len({e["MASTER_PORT"] for e in ranks}) == 1
    assert all(e["SSQ_LAUNCHER"] == "self-spawned" for e in ranks)


def test_spawn_ranks_propagates_failure(tmp_path):
    """A failing rank's exit code is the job's, and the other ranks are stopped."""
    import time as _time
    from shiftedscalequantization_amd.launch import spawn_ranks
    script = tmp_path / "rank.py"
    script.write_text("import os, sys, time\n"
                      "if os.environ['RANK'] == '1':\n    sys.exit(3)\n"
                      "time.sleep(60)\n")
    t0 = _time.time()
    assert spawn_ranks(str(script), [], 2, check_parent=False) == 3
    assert _time.time() - t0 < 30
    ok = tmp_path / "ok.py"
    ok.write_text("import os\nassert os.environ['WORLD_SIZE'] == '3'\n")
    assert spawn_ranks(str(ok), [], 3, check_parent=False) == 0


def test_no_spawn_under_external_launcher(monkeypatch):
    from shiftedscalequantization_amd import launch
    monkeypatch.setenv("WORLD_SIZE", "4")
    monkeypatch.delenv("SSQ_LAUNCH_DRYRUN", raising=False)
    called = []
    monkeypatch.setattr(launch, "spawn_ranks", lambda *a: called.append(a))
    launch.maybe_spawn("x.py", ["--gpus", "4"])
    monkeypatch.delenv("WORLD_SIZE")
    launch.maybe_spawn("x.py", ["--gpus", "1"])
    assert called == []


def test_grads_into_one_write_per_parameter():
    """Inside one grads_into context (one iteration's backward) each parameter's gradient
    slice may be written by one kernel only: a second producer would overwrite the first
    contribution, so _grad_dest raises; a new context starts afresh."""
    from shiftedscalequantization_amd import _capi as A
    from shiftedscalequantization_amd import kernels as K
    p, q = torch.zeros(6), torch.zeros(4)
    bucket = torch.zeros(10)
    into = {p.data_ptr(): bucket[:6], q.data_ptr(): bucket[6:]}
    for _ in range(2):
        with K.grads_into(into):
            d, written = K._grad_dest(p, 6, p.device)
            assert written and d.data_ptr() == bucket.data_ptr()
            K._grad_dest(q, 4, q.device)
            with pytest.raises(A.SSQError):
                K._grad_dest(p, 6, p.device)
    assert not K.GRAD_INTO


# ---- the first RCCL run (the driver's 8-GPU node), rehearsed on the host ------------------

def test_eight_rccl_ranks_map_to_distinct_devices(monkeypatch):
    """`bench.py --gpus 8 --dist-backend nccl` / `main_imagenet.py --gpus 8`: the self-spawner
    gives the 8 ranks LOCAL_RANK 0..7, and with 8 devices visible (mocked here) each rank
    binds cuda:LOCAL_RANK and initialises RCCL with that device -- no two ranks share a GPU.
    With fewer devices than ranks, RCCL is refused with a pointer to gloo."""
    import importlib
    import sys
    import torch.distributed as dist
    sys.path.insert(0, ROOT)
    for script, args in (("bench.py", ["--gpus", "8", "--dist-backend", "nccl"]),
                         ("main_imagenet.py", ["--gpus", "8", "--dist_backend", "nccl"])):
        parent, ranks = _dryrun(script, args)
        assert [e["LOCAL_RANK"] for e in ranks] == [str(r) for r in range(8)]
        mod = importlib.import_module(script[:-3])
        bound = []

        class _Stop(Exception):
            pass

        def init_pg(backend, device_id=None, **k):
            bound.append((backend, device_id))
            if script == "main_imagenet.py":
                raise _Stop()          # main() goes on to build the model: stop at RCCL

        monkeypatch.setattr(torch.cuda, "device_count", lambda: 8)
        monkeypatch.setattr(torch.cuda, "set_device", lambda d: None)
        monkeypatch.setattr(dist, "init_process_group", init_pg)
        for e in ranks:
            for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT"):
                monkeypatch.setenv(k, e[k])
            if script == "bench.py":
                monkeypatch.setattr(sys, "argv", [script] + args)
                mod.setup(mod.parse().dist_backend)
            else:
                with pytest.raises(_Stop):
                    mod.main(args)
        assert [b for b, _ in bound] == ["nccl"] * 8, bound
        assert [d for _, d in bound] == [torch.device("cuda", r) for r in range(8)], bound
        # 8 ranks over RCCL on a 4-GPU box: refused (gloo rehearses shared devices)
        monkeypatch.setattr(torch.cuda, "device_count", lambda: 4)
        with pytest.raises(SystemExit, match="gloo"):
            if script == "bench.py":
                mod.setup("nccl")
            else:
                mod.main(args)
    for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT"):
        monkeypatch.delenv(k, raising=False)


def test_collective_stays_outside_graph_capture(monkeypatch):
    """At world > 1 the reconstruction iteration is captured as two HIP graphs around the
    gradient bucket's all-reduce (_engine.IterationGraph): the body's kernels are captured,
    the collective never is -- RCCL's all-reduce runs eagerly between the two replays, in
    the iteration's order (pre replay, all-reduce, post replay).  Graph capture and the
    collective are mocked (host only); the bucket and the graph split are the product's."""
    import torch.distributed as dist
    from shiftedscalequantization_amd import parallel_dp as P
    from shiftedscalequantization_amd.quant import _engine as E
    state, log = {"capturing": False}, []

    class Graph:
        def __init__(self):
            self.body = None

        def pool(self):
            return None

        def replay(self):
            log.append(("replay", self.body))

    class capture:
        def __init__(self, g, pool=None):
            self.g = g

        def __enter__(self):
            state["capturing"] = True
            state["graph"] = self.g

        def __exit__(self, *exc):
            state["capturing"] = False

    def all_reduce(t, op=None):
        assert not state["capturing"], "collective inside a graph capture"
        log.append(("all_reduce", t.numel()))

    monkeypatch.setattr(torch.cuda, "CUDAGraph", Graph)
    monkeypatch.setattr(torch.cuda, "graph", capture)
    monkeypatch.setattr(dist, "all_reduce", all_reduce)
    monkeypatch.setattr(P, "world", lambda: 8)
    a, b = torch.zeros(5, requires_grad=True), torch.zeros(3, requires_grad=True)
    bucket = P.GradBucket([a, b])
    a.grad, b.grad = torch.ones(5), torch.ones(3)
    bucket.allreduce_()                       # builds the flat bucket (8 elements)
    assert bucket.active and log == [("all_reduce", 8)]
    log.clear()

    def pre():
        assert state["capturing"]
        state["graph"].body = "pre"

    def post():
        assert state["capturing"]
        state["graph"].body = "post"

    ig = E.IterationGraph(pre, post, bucket, {})
    assert len(ig.graphs) == 2 and log == []
    for _ in range(3):
        ig.replay()
    assert log == [("replay", "pre"), ("all_reduce", 8), ("replay", "post")] * 3, log
    # world 1: one graph, no collective
    monkeypatch.setattr(P, "world", lambda: 1)
    log.clear()
    ig1 = E.IterationGraph(pre, lambda: None, P.GradBucket([a]), {})
    ig1.replay()
    assert len(ig1.graphs) == 1 and log == [("replay", "pre")]
