"""Data-parallel reconstruction (§8(e), config 5's sharded path) at world size 2.

Two ranks share the box's one GPU over gloo (RCCL needs one GPU per rank; the bucket /
collective logic is backend-independent).  Each rank reconstructs on its half of the
calibration data.  Checked, bit for bit:
  * every iteration's all-reduced bucket is identical on both ranks and equals the sum
    of the two ranks' local buckets (the reference's SUM, block_recon.py:100-102);
  * the learned parameters (shift logits alpha; AdaRound V; act deltas) are identical on
    both ranks after the loop -- replicated, as the all-reduce design assumes;
  * they equal a single-process replay that feeds Adam the summed gradients from the
    same starting point (the "1-rank run fed the summed gradient of both shards");
  * the act deltas initialised on different shards differ before, and are identical
    after, synchorize_activation_statistics (their mean);
  * after the eager warm-up the iterations replay HIP graphs split around the collective
    (quant._engine.IterationGraph), so all of the above holds for the graph path.
"""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _run_world2(mode, tmp_path):
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    port = _free_port()
    procs, outs = [], []
    for r in range(2):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE="2", LOCAL_RANK="0",
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        out = str(tmp_path / f"{mode}_r{r}.npz")
        outs.append(out)
        procs.append(subprocess.Popen([sys.executable, os.path.join(HERE, "dp_worker.py"), mode, out],
                                      env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT))
    logs = []
    try:
        for p in procs:
            logs.append(p.communicate(timeout=100)[0].decode(errors="replace"))
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    for p, log in zip(procs, logs):
        assert p.returncode == 0, log[-3000:]
    return [dict(np.load(o)) for o in outs]


def _check_buckets(r0, r1):
    # the iterations after the eager warm-up replay the two graphs around the collective
    assert int(r0["split_replays"][0]) > 0 and int(r1["split_replays"][0]) > 0
    n = int(r0["n_rec"][0])
    assert n == int(r1["n_rec"][0]) and n > 0
    for k in range(n):
        red0, red1 = r0[f"rec{k}_reduced"], r1[f"rec{k}_reduced"]
        np.testing.assert_array_equal(red0, red1)
        np.testing.assert_array_equal(red0, r0[f"rec{k}_local"] + r1[f"rec{k}_local"])
        assert not np.array_equal(r0[f"rec{k}_local"], r1[f"rec{k}_local"])  # different shards
    return [r0[f"rec{k}_reduced"] for k in range(n)]


@pytest.mark.parametrize("bias_cal", [False, True])
def test_fused_recon_world2_replicated(tmp_path, bias_cal):
    """bias_cal: gamma^z / phi^z in the bucket too.  The deferred loss / gamma^z / phi^z
    finalizes stay on at world 2: the backward kernels write alpha, gamma^z and phi^z straight
    into their bucket slices (K.grads_into; counted by K.INTO_WRITES)."""
    from shiftedscalequantization_amd.quant._engine import SsqAdam
    r0, r1 = _run_world2("fused_bc" if bias_cal else "fused", tmp_path)
    reduced = _check_buckets(r0, r1)
    convs = ("conv1", "conv2", "downsample")
    keys = [(n, k) for n in convs for k in (("alpha", "gamma", "phi") if bias_cal else ("alpha",))]
    for n, k in keys:
        np.testing.assert_array_equal(r0[f"{n}_{k}0"], r1[f"{n}_{k}0"])
        np.testing.assert_array_equal(r0[f"{n}_{k}"], r1[f"{n}_{k}"])
    # every iteration after the bucket is built: one write per parameter, per rank
    assert int(r0["into_writes"][0]) >= len(keys) * 2, int(r0["into_writes"][0])
    # single-process replay: Adam (lr 1e-3) fed the summed buckets from the same start
    params = [torch.nn.Parameter(torch.as_tensor(r0[f"{n}_{k}0"]).cuda()) for n, k in keys]
    opt = SsqAdam(params, lr=1e-3)
    sizes = [p.numel() for p in params]
    for flat in reduced:
        parts = np.split(flat, np.cumsum(sizes)[:-1])
        for p, g in zip(params, parts):
            p.grad = torch.as_tensor(g).view_as(p).cuda()
        opt.step()
    for (n, k), p in zip(keys, params):
        np.testing.assert_array_equal(p.detach().cpu().numpy(), r0[f"{n}_{k}"], err_msg=n + k)
    np.testing.assert_array_equal(r0["final_losses"] != r1["final_losses"], [True, True])
    if bias_cal:
        assert any(np.any(r0[f"{n}_gamma"] != 1.0) for n in convs)


def test_fused_recon_world2_deferral_bit_identical(tmp_path):
    """World 2 with bias_cal: the loop with the deferred finalizes writing into the bucket
    and the loop finalizing each gradient by its own launch (DEFER_FINALIZE off) give
    bit-identical buckets, parameters and losses."""
    on = _run_world2("fused_bc", tmp_path)
    off = _run_world2("fused_bc_nodefer", tmp_path)
    assert int(on[0]["into_writes"][0]) > 0 and int(off[0]["into_writes"][0]) == 0
    for a, b in zip(on, off):
        assert int(a["n_rec"][0]) == int(b["n_rec"][0])
        for k in a:
            if k in ("into_writes",):
                continue
            np.testing.assert_array_equal(a[k], b[k], err_msg=k)


def test_brecq_world2_replicated(tmp_path):
    r0, r1 = _run_world2("brecq", tmp_path)
    _check_buckets(r0, r1)
    for n in ("conv1", "conv2", "downsample"):
        np.testing.assert_array_equal(r0[n + "_V"], r1[n + "_V"], err_msg=n)
    assert not np.array_equal(r0["a_delta_local"], r1["a_delta_local"])
    np.testing.assert_array_equal(r0["a_delta0"], r1["a_delta0"])
    np.testing.assert_allclose(r0["a_delta0"], (r0["a_delta_local"] + r1["a_delta_local"]) / 2,
                               rtol=1e-6)
    np.testing.assert_array_equal(r0["a_delta"], r1["a_delta"])


def test_validation_world2_whole_set_top1(tmp_path):
    """(f3) sharded validation: each rank sees only its half of the val batches, and both
    return the reference's whole-set top-1 (the (correct, total) all-reduce)."""
    r0, r1 = _run_world2("validate", tmp_path)
    g = np.load(os.path.join(HERE, "golden", "validate_w2a4.npz"))
    assert int(r0["n_local"][0]) + int(r1["n_local"][0]) == len(g["labels"])
    assert int(r0["n_local"][0]) != len(g["labels"])
    assert float(r0["top1"][0]) == float(g["top1"][0])
    assert float(r1["top1"][0]) == float(g["top1"][0])


@pytest.mark.timeout(600)
def test_bench_self_launches_two_ranks():
    """`python bench.py --gpus 2` with no launcher in the environment starts its own two
    rank processes (launch.py; the reference's mp.spawn, Brecq/main_imagenet_dist.py:268-271),
    and rank 0's line reports what the process group saw.  Over gloo here: RCCL needs one
    GPU per rank and this box has one, so the two ranks share cuda:0."""
    import json
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    root = os.path.dirname(HERE)
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2",
                        "--dist-backend", "gloo", "--steps", "2", "--warmup", "1",
                        "--no-cpu-baseline", "--no-validate", "--recon-iters", "8"],
                       env=env, cwd=root, capture_output=True, text=True, timeout=540)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-4000:])
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]          # rank 0 only
    out = lines[0]
    assert out["n_gpus"] == 2 and out["config"]["parallelism"] == "dp2"
    assert out["launch"] == {"launcher": "self-spawned", "world_size_backend": 2,
                             "allreduce_backend": "gloo",
                             "devices_visible": torch.cuda.device_count()}
    assert out["recon"]["n_gpus"] == 2 and out["value"] > 0
    print(json.dumps({"self_launch_world2": {k: out[k] for k in ("value", "ms_per_step")},
                      "recon_all_blocks_it_s": out["recon"].get("resnet18_all_blocks_iters_per_s")}))
