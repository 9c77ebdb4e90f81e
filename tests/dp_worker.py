"""One rank of the world-size-2 data-parallel reconstruction tests (tests/test_dp_gpu.py).

Started twice by the test (RANK 0 / 1, MASTER_ADDR 127.0.0.1) on the one GPU of the box:
gloo moves the device gradient bucket through the host, which exercises the same
GradBucket / all-reduce path RCCL runs on an 8-GPU node.  Each rank takes its contiguous
half of the fixture's calibration data (parallel_dp.shard_rows), runs the loop, and
writes what the test compares: the learned parameters, their values before the loop, and
every iteration's (local, all-reduced) gradient bucket (parallel_dp.RECORD).

    python tests/dp_worker.py {fused|fused_bc|fused_bc_nodefer|brecq|validate} OUT.npz
"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, HERE)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

FUSED_ITERS, FUSED_BS = 12, 4
BRECQ_ITERS, BRECQ_BS = 8, 4


def dev(a):
    return torch.as_tensor(np.asarray(a)).cuda()


def host(t):
    return t.detach().float().cpu().numpy().copy()


def run_fused_bc(out):
    run_fused(out, bias_cal=True)


def run_fused_bc_nodefer(out):
    import importlib
    # the module (quant/__init__ re-exports a function of the same name)
    LRF = importlib.import_module("shiftedscalequantization_amd.quant.layer_recon_fused_shiftedScale")
    LRF.DEFER_FINALIZE = False
    run_fused(out, bias_cal=True)


def run_fused(out, bias_cal=False):
    from conftest import load_golden
    import test_recon_gpu as T
    from shiftedscalequantization_amd import quant as Q
    from shiftedscalequantization_amd.parallel_dp import shard_rows
    from shiftedscalequantization_amd.quant.layer_recon_fused_shiftedScale import \
        block_recon_fused_shiftedScale
    g = load_golden("recon_fused")
    qnn = T.build_qnn(Q, {})
    block = qnn.model[3]
    T.load_block(Q, g, block)
    lo, hi = shard_rows(len(g["cached_inp"]))
    block.cached_inp_features = [dev(g["cached_inp"][lo:hi])]
    block.cached_out_features = [dev(g["cached_out"][lo:hi])]
    convs = ("conv1", "conv2", "downsample")

    def hook(i):
        if i == 0:
            for n in convs:
                m = getattr(block, n)
                out[n + "_alpha0"] = host(m.weight_quantizer.alpha)
                out[n + "_gamma0"], out[n + "_phi0"] = host(m.alpha_out), host(m.beta_out)

    from shiftedscalequantization_amd import kernels as K
    K.INTO_WRITES[0] = 0
    torch.manual_seed(1005)
    res = block_recon_fused_shiftedScale(block, FUSED_ITERS, (0.01, 0.1), qnn, None, verbose=False,
                                         iter_hook=hook, batch_size=FUSED_BS, bias_cal=bias_cal)
    out["final_losses"] = np.array(res, np.float64)
    out["into_writes"] = np.array([K.INTO_WRITES[0]])
    for n in convs:
        m = getattr(block, n)
        out[n + "_alpha"] = host(m.weight_quantizer.alpha)
        out[n + "_gamma"], out[n + "_phi"] = host(m.alpha_out), host(m.beta_out)


def run_brecq(out):
    from conftest import load_golden
    import test_recon_gpu as T
    from shiftedscalequantization_amd import quant as Q
    from shiftedscalequantization_amd.parallel_dp import shard_rows
    g = load_golden("recon_brecq")
    qnn = T.build_qnn(Q, g)
    block = qnn.model[3]
    lo, hi = shard_rows(len(g["cali"]))
    cali = dev(g["cali"][lo:hi])
    convs = ("conv1", "conv2", "downsample")
    torch.manual_seed(1005)
    Q.block_reconstruction(qnn, block, cali, batch_size=BRECQ_BS, iters=BRECQ_ITERS, weight=0.01,
                           asym=True, b_range=(20, 2), warmup=0.2, act_quant=False, opt_mode="mse")
    for n in convs:
        out[n + "_V"] = host(getattr(block, n).weight_quantizer.alpha)
    # act phase: init on this rank's shard, all-average (Brecq/main_imagenet_dist.py:210-211)
    qnn.set_quant_state(True, True)
    with torch.no_grad():
        qnn(cali[:8])
    aqs = [block.act_quantizer] + [getattr(block, n).act_quantizer for n in convs
                                   if getattr(block, n).act_quantizer.delta is not None]
    out["a_delta_local"] = np.array([float(q.delta) for q in aqs], np.float32)
    qnn.synchorize_activation_statistics()
    out["a_delta0"] = np.array([float(q.delta) for q in aqs], np.float32)
    qnn.disable_network_output_quantization()
    torch.manual_seed(1005)
    Q.block_reconstruction(qnn, block, cali, batch_size=BRECQ_BS, iters=BRECQ_ITERS, act_quant=True,
                           opt_mode="mse", lr=4e-4, p=2.4)
    out["a_delta"] = np.array([float(q.delta) for q in aqs], np.float32)


def run_validate(out):
    """(f3) + (e): each rank validates its contiguous share of the fixture's val batches;
    cli.validate_model all-reduces (correct, total) (Brecq/main_imagenet_dist.py:114-124)."""
    import test_recon2_gpu as T2
    from shiftedscalequantization_amd import cli, quant as Q
    from shiftedscalequantization_amd.parallel_dp import shard_rows
    g = np.load(os.path.join(HERE, "golden", "validate_w2a4.npz"))
    qnn = T2.tiny_net2(Q, g)
    qnn.set_quant_state(True, True)
    with torch.no_grad():
        qnn(dev(g["cali"])[:8])
    qnn.disable_network_output_quantization()
    loader = T2._val_loader(g)
    lo, hi = shard_rows(len(loader))
    out["n_local"] = np.array([sum(int(t.numel()) for _, t in loader[lo:hi])])
    out["top1"] = np.array([cli.validate_model(loader[lo:hi], qnn)], np.float64)


def main():
    mode, path = sys.argv[1], sys.argv[2]
    torch.cuda.set_device(0)
    torch.backends.cudnn.benchmark = False
    torch.backends.cudnn.deterministic = True
    dist.init_process_group("gloo")
    from shiftedscalequantization_amd import parallel_dp as P
    P.RECORD = []
    out = {"rank": np.array([dist.get_rank()])}
    {"fused": run_fused, "fused_bc": run_fused_bc, "fused_bc_nodefer": run_fused_bc_nodefer,
     "brecq": run_brecq, "validate": run_validate}[mode](out)
    torch.cuda.synchronize()
    for k, (kind, local, reduced) in enumerate(P.RECORD):
        out[f"rec{k}_local"] = local.cpu().numpy()
        out[f"rec{k}_reduced"] = reduced.cpu().numpy()
    out["n_rec"] = np.array([len(P.RECORD)])
    from shiftedscalequantization_amd.quant._engine import GRAPH_REPLAYS
    out["split_replays"] = np.array([GRAPH_REPLAYS["split"]])
    np.savez(path, **out)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
