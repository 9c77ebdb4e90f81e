"""Command-line flags of the calibration driver (main_imagenet.py).

Union of the README's command (README.md:20: --device_gpu --arch --n_bits_w --n_bits_a
--weight --bias_cal --bias_ch_quant), the shifted-scale driver's flags (common.py:19-75)
and BRECQ's (Brecq/main_imagenet.py:135-169).  Boolean flags keep the reference's
`type=bool` parsing (any non-empty string, "False" included, is True) so existing
command lines behave identically.
"""
import argparse
import os
import random

import numpy as np
import torch


def build_parser():
    p = argparse.ArgumentParser(description='running parameters',
                                formatter_class=argparse.ArgumentDefaultsHelpFormatter)
    # general
    p.add_argument('--seed', default=1005, type=int)
    p.add_argument('--arch', default='resnet18', type=str,
                   choices=['resnet18', 'resnet34', 'resnet50', 'mobilenetv2', 'regnetx_600m',
                            'regnetx_3200m', 'mnasnet'])
    p.add_argument('--batch_size', default=64, type=int)
    p.add_argument('--workers', default=4, type=int)
    p.add_argument('--data_path', default='', type=str,
                   help='directory with cali.pt / val.pt tensors; empty -> synthetic data')
    p.add_argument('--checkpoint', default='', type=str, help='FP state_dict (weights_only load)')
    p.add_argument('--device_gpu', default='cuda:0', type=str)
    p.add_argument('--run_device', default='', type=str, help='alias of --device_gpu (common.py)')
    # quantization
    p.add_argument('--n_bits_w', default=2, type=int)
    p.add_argument('--channel_wise', default=True, type=bool)
    p.add_argument('--n_bits_a', default=4, type=int)
    p.add_argument('--act_quant', default=True, type=bool)
    p.add_argument('--disable_8bit_head_stem', default=False, type=bool)
    p.add_argument('--test_before_calibration', default=False, type=bool)
    p.add_argument('--w_scale_method', default='mse', type=str)
    p.add_argument('--a_scale_method', default='mse', type=str)
    # weight calibration
    p.add_argument('--num_samples', default=1024, type=int)
    p.add_argument('--iters_w', default=20000, type=int)
    p.add_argument('--weight', default=0.01, type=float,
                   help='lambda of the rounding and group (shift) policy')
    p.add_argument('--sym', default=False, type=bool)
    p.add_argument('--b_start', default=20, type=int)
    p.add_argument('--b_end', default=2, type=int)
    p.add_argument('--warmup', default=0.2, type=float)
    p.add_argument('--step', default=20, type=int)
    # activation calibration
    p.add_argument('--iters_a', default=5000, type=int)
    p.add_argument('--lr', default=4e-4, type=float)
    p.add_argument('--p', default=2.4, type=float)
    # shifted-scale (README "Key Options")
    p.add_argument('--bias_cal', default=False, type=bool,
                   help='learn the output-channel scale gamma^z and offset phi^z')
    p.add_argument('--bias_ch_quant', default=False, type=bool,
                   help='learn the input-channel shift group R (fused shifted-scale recon)')
    p.add_argument('--shift_iters', default=625, type=int,
                   help='iterations of the fused shifted-scale recon (ShiftedScaleQuant.py:386)')
    p.add_argument('--shift_targets', default='0.96875,1.03125,1.0', type=str)
    p.add_argument('--mse_level', default=1, type=int)
    p.add_argument('--mse_threshold', default=1.0, type=float)
    p.add_argument('--shift_quant_mode', default='max', type=str)
    p.add_argument('--test', default=False, type=bool, help='ChannelQuantMSE path (channelShift_wMSE)')
    p.add_argument('--skip_test', default=False, type=bool)
    p.add_argument('--keep_features_on_host', default=False, type=bool)
    p.add_argument('--deterministic', default=1, type=int,
                   help='1 (reference): deterministic MIOpen conv solvers; 0: fastest solvers')
    # data parallel: one process per GPU, spawned by main_imagenet.py itself with --gpus N
    # (the reference's mp.spawn, Brecq/main_imagenet_dist.py:268-271) or by an external
    # torch.distributed.run
    p.add_argument('--gpus', default=1, type=int,
                   help='ranks to spawn on this node (one per GPU) when no launcher set WORLD_SIZE')
    p.add_argument('--dist_backend', default='nccl', type=str,
                   help="torch.distributed backend for world > 1: 'nccl' (= RCCL over xGMI); "
                        "'gloo' rehearses several ranks on one GPU")
    return p


def parse_args(argv=None):
    a = build_parser().parse_args(argv)
    if a.run_device:
        a.device_gpu = a.run_device
    return a


def seed_all(seed=1029, deterministic=True):
    """common.py:77-85.  deterministic=True (the reference's setting) restricts MIOpen to
    deterministic convolution solvers -- for some stride-2 / 1x1 weight gradients that is a
    naive kernel; False lets MIOpen pick its fastest solvers (the ssq kernels are
    deterministic either way)."""
    random.seed(seed)
    os.environ['PYTHONHASHSEED'] = str(seed)
    np.random.seed(seed)
    torch.manual_seed(seed)
    if torch.cuda.is_available():
        torch.cuda.manual_seed_all(seed)
    torch.backends.cudnn.benchmark = False
    torch.backends.cudnn.deterministic = bool(deterministic)


def accuracy(output, target, topk=(1,)):
    """common.py:128-142."""
    with torch.no_grad():
        maxk = max(topk)
        bs = target.size(0)
        _, pred = output.topk(maxk, 1, True, True)
        correct = pred.t().eq(target.view(1, -1).expand_as(pred.t()))
        return [correct[:k].reshape(-1).float().sum(0, keepdim=True).mul_(100.0 / bs) for k in topk]


def get_train_samples(train_loader, num_samples):
    """common.py:144-150."""
    data = []
    for batch in train_loader:
        data.append(batch[0])
        if len(data) * batch[0].size(0) >= num_samples:
            break
    return torch.cat(data, dim=0)[:num_samples]


@torch.no_grad()
def validate_model(val_loader, model, device=None, print_result=False):
    """common.py:152-221: top-1 over (images, target) batches.  With several ranks each
    validates its own shard of the validation set and the (correct, total) sums are
    all-reduced (Brecq/main_imagenet_dist.py:114-124), so every rank returns the
    whole-set top-1."""
    from .parallel_dp import all_sum_
    from .quant.quant_layer import frozen_weight_cache
    device = next(model.parameters()).device if device is None else device
    model.eval()
    sums = torch.zeros(2, dtype=torch.float64, device=device)
    # every layer's W_hat is quantized once per pass, not once per batch (bit-identical)
    with frozen_weight_cache():
        for images, target in val_loader:
            out = model(images.to(device))
            sums[0] += (out.argmax(1) == target.to(device)).sum()
            sums[1] += target.numel()
    all_sum_(sums)
    correct, total = sums.tolist()
    acc = 100.0 * correct / max(total, 1)
    if print_result:
        print(f' * Acc@1 {acc:.3f}')
    return acc
