#!/bin/bash
# Rehearse the N > 1 bench path on a 1-GPU box: 2 ranks sharing cuda:0 over gloo (the
# driver's 8-GPU runs use RCCL).  Usage (via gpurun): bash tools/dist_rehearsal.sh <tag>
TAG=${1:-run}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 5 --warmup 2 --dist-backend gloo --recon-iters 30 --n-cali 256 > $OUT/dist2_$TAG.log 2>&1 || { echo "dist rehearsal failed"; tail -30 $OUT/dist2_$TAG.log; exit 1; }
grep '^{' $OUT/dist2_$TAG.log | tail -1
