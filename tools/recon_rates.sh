#!/bin/bash
# GPU tests + BRECQ and fused shifted-scale recon iteration rates.  Usage: bash tools/recon_rates.sh <tag>
TAG=${1:-run}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
timeout -k 10 600 python -m pytest tests -m gpu -q -x > $OUT/pytest_$TAG.log 2>&1
rc=$?
tail -3 $OUT/pytest_$TAG.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python tools/brecq_bench.py > $OUT/brecq_$TAG.log 2>&1 || { tail -20 $OUT/brecq_$TAG.log; exit 1; }
tail -1 $OUT/brecq_$TAG.log
timeout -k 10 300 python -c "import torch, json; from shiftedscalequantization_amd.recon_bench import run_recon_bench; print(json.dumps(run_recon_bench(torch.device('cuda'), 1, 0)['iters_per_s']))" > $OUT/fused_$TAG.log 2>&1 || { tail -20 $OUT/fused_$TAG.log; exit 1; }
tail -1 $OUT/fused_$TAG.log
