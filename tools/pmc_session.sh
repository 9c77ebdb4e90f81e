#!/bin/bash
# Two PMC passes (FETCH_SIZE, WRITE_SIZE) over a short q/dq-only bench, then per-launch
# HBM bytes.  Usage (via gpurun): bash tools/pmc_session.sh <tag>
TAG=${1:-run}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch_$TAG -o f -- python3 $R/bench.py --no-recon --no-cpu-baseline --steps 3 --warmup 1 > $OUT/pmc_fetch_$TAG.log 2>&1 || { echo "fetch pass failed"; tail -20 $OUT/pmc_fetch_$TAG.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write_$TAG -o w -- python3 $R/bench.py --no-recon --no-cpu-baseline --steps 3 --warmup 1 > $OUT/pmc_write_$TAG.log 2>&1 || { echo "write pass failed"; tail -20 $OUT/pmc_write_$TAG.log; exit 1; }
python3 $R/tools/pmc_traffic.py $OUT/pmc_fetch_$TAG $OUT/pmc_write_$TAG $OUT/pmc_traffic_$TAG.json
