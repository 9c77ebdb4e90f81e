#!/bin/bash
# A/B of the K13 epilogue folded into conv2's im2col GEMM (SSQ_EPI_GEMM, ResNet-18 layer3/4
# BasicBlocks) in bench.py's recon loops, ABAB on one box: per-block iterations/s.
TAG=${1:-epi}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
for V in 1 0 1 0; do
  SSQ_EPI_GEMM=$V timeout -k 10 300 python bench.py --no-cpu-baseline --no-validate --steps 3 --warmup 1 > $OUT/epi_${TAG}_$V.log 2>&1 || { echo "bench $V failed"; tail -5 $OUT/epi_${TAG}_$V.log; exit 1; }
  tail -1 $OUT/epi_${TAG}_$V.log | python -c "import json,sys; d=json.loads(sys.stdin.read())['recon']; print('SSQ_EPI_GEMM=$V', json.dumps(d['iters_per_s']), d['resnet18_all_blocks_iters_per_s'])"
done
