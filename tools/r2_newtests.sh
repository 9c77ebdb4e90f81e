#!/bin/bash
# Round-2 new GPU tests only (fast turnaround).  Usage (via gpurun): bash tools/r2_newtests.sh TAG
TAG=${1:-run}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
export SSQ_PARITY_LOG=$OUT/parity_$TAG.jsonl
rm -f $SSQ_PARITY_LOG
timeout -k 10 500 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_kernels_gpu.py -k "prepared or hard_weights" \
  > $OUT/newtests_k_$TAG.log 2>&1
rc=$?
tail -5 $OUT/newtests_k_$TAG.log
if [ $rc -ne 0 ]; then echo "kernel tests rc=$rc"; exit $rc; fi
timeout -k 10 120 python -u tools/adashift_bench.py > $OUT/adashift_bench_$TAG.log 2>&1 || { echo "adashift bench failed"; tail -20 $OUT/adashift_bench_$TAG.log; exit 1; }
cat $OUT/adashift_bench_$TAG.log
if [ -n "$RECON" ]; then
timeout -k 10 500 python -u -m pytest -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_recon2_gpu.py tests/test_dp_gpu.py > $OUT/newtests_r_$TAG.log 2>&1
rc=$?
tail -15 $OUT/newtests_r_$TAG.log
exit $rc
fi
