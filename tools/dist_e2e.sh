#!/bin/bash
# Config 5's sharded path end to end on a 1-GPU box: main_imagenet.py on RegNetX-3200M W2A4
# (fused shifted-scale recon with bias_cal on every block, BRECQ act phase) as 2 ranks
# sharing cuda:0 over gloo (the driver's 8-GPU runs use RCCL), synthetic calibration data
# sharded per rank, short loops.  Each rank prints whether its calibrated model is
# bit-identical to the other's.  Usage (via gpurun): bash tools/dist_e2e.sh <tag>
TAG=${1:-run}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 main_imagenet.py --arch regnetx_3200m --n_bits_w 2 --n_bits_a 4 --bias_ch_quant True --bias_cal True --num_samples 128 --shift_iters 40 --iters_w 40 --iters_a 40 --dist_backend gloo > $OUT/dist_e2e_$TAG.log 2>&1 || { echo "dist e2e failed"; tail -30 $OUT/dist_e2e_$TAG.log; exit 1; }
grep "replicated\|calibration finished" $OUT/dist_e2e_$TAG.log | cut -c1-300
