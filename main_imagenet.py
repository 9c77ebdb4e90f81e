"""Shifted-scale PTQ calibration driver (the README's entry point, README.md:20).

    python main_imagenet.py --device_gpu=cuda:0 --arch=resnet18 --n_bits_w=2 --n_bits_a=4 \
        --weight=1.0 --bias_cal=True --bias_ch_quant=True [--data_path DIR] [--checkpoint FP.pt]

Flow (the README flags mapped onto the snapshot's code):
  1. QuantModel(arch) with W n_bits_w per-channel / A n_bits_a per-tensor; 8-bit stem/head;
     weight delta/zp initialised on the first 64 calibration samples.
  2. --bias_ch_quant: every residual block is reconstructed with the fused shifted-scale
     loop (ChannelQuant 'adaShift', learns the input-channel shift group R); --bias_cal
     additionally learns gamma^z / phi^z.  Otherwise BRECQ AdaRound reconstruction.
  3. --act_quant: activation deltas initialised and reconstructed BRECQ-style (LSQ, p=2.4).
  4. Top-1 on --data_path/val.pt if present ("Weight quantization accuracy",
     "Full quantization (W{w}A{a}) accuracy"); otherwise the reconstruction losses.
Data: --data_path may hold cali.pt ([N,3,224,224] float) and val.pt ((images, labels));
without it synthetic N(0,1) calibration images are used (no network access here).
Multi-GPU: `--gpus N` spawns N rank processes (as the reference's mp.spawn,
Brecq/main_imagenet_dist.py:268-271), or launch with torch.distributed.run; each rank
calibrates on its shard of the calibration set and the per-iteration gradients are
all-reduced over RCCL.
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

if __name__ == '__main__':
    # before torch is imported: the parent of the spawned ranks never loads the HIP runtime
    from shiftedscalequantization_amd.launch import maybe_spawn
    maybe_spawn(os.path.abspath(__file__))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from shiftedscalequantization_amd import drivers as D  # noqa: E402
from shiftedscalequantization_amd.cli import parse_args, seed_all, validate_model  # noqa: E402
from shiftedscalequantization_amd.parallel_dp import replicated, shard_rows  # noqa: E402
from shiftedscalequantization_amd.quant import QuantModule  # noqa: E402


def load_data(args, device):
    cali = val = None
    if args.data_path and os.path.exists(os.path.join(args.data_path, 'cali.pt')):
        cali = torch.load(os.path.join(args.data_path, 'cali.pt'), weights_only=True)
    if args.data_path and os.path.exists(os.path.join(args.data_path, 'val.pt')):
        val = torch.load(os.path.join(args.data_path, 'val.pt'), weights_only=True)
    if cali is None:
        g = torch.Generator().manual_seed(args.seed)
        cali = torch.randn(args.num_samples, 3, 224, 224, generator=g)
    lo, hi = shard_rows(len(cali))
    return cali[lo:hi].to(device), val


def val_loader(val, bs=256):
    """This rank's shard of the validation set in batches (validate_model all-reduces the
    per-rank sums)."""
    if val is None:
        return None
    images, labels = val
    lo, hi = shard_rows(len(images))
    images, labels = images[lo:hi], labels[lo:hi]
    return [(images[i:i + bs], labels[i:i + bs]) for i in range(0, len(images), bs)]


def main(argv=None):
    args = parse_args(argv)
    world = int(os.environ.get('WORLD_SIZE', '1'))
    if world > 1:
        # one process per GPU; ranks beyond the visible GPUs share them (gloo rehearsals)
        local = int(os.environ.get('LOCAL_RANK', '0'))
        ndev = torch.cuda.device_count()
        if args.dist_backend == 'nccl' and world > ndev:
            raise SystemExit(f'main_imagenet.py: {world} ranks over RCCL need {world} GPUs, {ndev} '
                             f'visible (rehearse with --dist_backend gloo: ranks then share devices)')
        device = torch.device('cuda', local % max(ndev, 1))
        torch.cuda.set_device(device)
        if args.dist_backend == 'nccl':
            dist.init_process_group('nccl', device_id=device)
        else:
            dist.init_process_group(args.dist_backend)
    else:
        device = torch.device(args.device_gpu)
    seed_all(args.seed, deterministic=bool(args.deterministic))
    cali, val = load_data(args, device)
    loader = val_loader(val)
    t0 = time.time()
    qnn = D.build_qnn(args.arch, args.n_bits_w, args.n_bits_a, args.channel_wise, args.w_scale_method,
                      args.a_scale_method, device, args.checkpoint, args.disable_8bit_head_stem)
    if args.test:
        # the shipped default (`ShiftedScaleQuant.py --test=True` -> channelShift_wMSE,
        # :119-183): input-channel scales by the ChannelQuantMSE range test, no recon loop
        shifts = [float(s) for s in args.shift_targets.split(',')]
        fc = [n for n, m in qnn.named_modules() if isinstance(m, QuantModule)][-1]
        D.channelShift_wMSE(qnn, cali, level=args.mse_level, threshold=args.mse_threshold,
                            opt_mode=args.shift_quant_mode, shiftTarget=shifts,
                            layerDisabled=['.' + fc])
        torch.cuda.synchronize(device)
        acc = validate_model(loader, qnn) if loader is not None else None
        print(f'channelShift_wMSE (level {args.mse_level}, threshold {args.mse_threshold}) '
              f'finished in {time.time() - t0:.1f}s; accuracy of qnn_hard: {acc}')
        if world > 1:
            dist.destroy_process_group()
        return qnn
    qnn.set_quant_state(True, False)
    with torch.no_grad():
        qnn(cali[:64])
    bs = 32
    report = {}
    phases = {'init': time.time() - t0}
    t_phase = time.time()
    if args.bias_ch_quant:
        shifts = [float(s) for s in args.shift_targets.split(',')]
        blocks = D.block_paths(qnn)
        D.build_ShiftedChannelQuant(qnn, blocks, '', shiftTarget=shifts, skipShiftLayer=[])
        qnn.set_quant_state(False, False)
        for path in blocks:
            D.cache_block_features(qnn, path, cali, bs, device)
            D.set_quant_state_block(qnn, [path], '', True)
            res = D.QuantRecursiveShiftRecon(qnn, [path], qnn, loader, iters=args.shift_iters,
                                             lmda=0.1 * args.weight, lmdaR=0.01 * args.weight,
                                             bias_cal=args.bias_cal)
            report.update(res)
            D.find_module(qnn, path).clear_cached_features()
        # the remaining single layers (fc) with BRECQ AdaRound
        last = [m for m in qnn.modules() if isinstance(m, QuantModule)][-1]
        from shiftedscalequantization_amd.quant import layer_reconstruction
        layer_reconstruction(qnn, last, cali, batch_size=bs, iters=args.iters_w, weight=0.01,
                             asym=True, b_range=(args.b_start, args.b_end), warmup=args.warmup,
                             act_quant=False, opt_mode='mse')
    else:
        D.recon_model(qnn, qnn, cali_data=cali, iters=args.iters_w, weight=args.weight, asym=True,
                      b_range=(args.b_start, args.b_end), warmup=args.warmup, act_quant=False,
                      opt_mode='mse', batch_size=bs)
    torch.cuda.synchronize(device)
    phases['weight_recon'] = time.time() - t_phase
    t_phase = time.time()
    qnn.set_quant_state(weight_quant=True, act_quant=False)
    if loader is not None:
        print('Weight quantization accuracy: {}'.format(validate_model(loader, qnn)))
    if args.act_quant:
        qnn.set_quant_state(True, True)
        with torch.no_grad():
            qnn(cali[:64])
        if world > 1:
            # each rank initialised its act deltas on its own shard: all-average them
            # (Brecq/main_imagenet_dist.py:210-211) so the act phase starts replicated
            qnn.synchorize_activation_statistics()
        qnn.disable_network_output_quantization()
        D.recon_model(qnn, qnn, cali_data=cali, iters=args.iters_a, act_quant=True, opt_mode='mse',
                      lr=args.lr, p=args.p, batch_size=bs)
        qnn.set_quant_state(weight_quant=True, act_quant=True)
        torch.cuda.synchronize(device)
        phases['act_recon'] = time.time() - t_phase
        if loader is not None:
            print('Full quantization (W{}A{}) accuracy: {}'.format(args.n_bits_w, args.n_bits_a,
                                                                   validate_model(loader, qnn)))
    print(f'calibration finished in {time.time() - t0:.1f}s '
          f'({", ".join(f"{k} {v:.1f}s" for k, v in phases.items())}); block rec losses: '
          f'{ {k: v for k, v in report.items()} }')
    if world > 1:
        # the calibrated model (learned shift logits, AdaRound V, gamma^z/phi^z, act deltas)
        # must be bit-identical on every rank
        print(f'rank {dist.get_rank()}/{world}: calibrated model replicated across ranks: '
              f'{replicated(qnn)}')
        dist.destroy_process_group()
    return qnn


if __name__ == '__main__':
    main()
