#!/bin/bash
# r5k5 A/B: the iteration-start launch with the prepared forward's (K5p) workgroups first in
# the grid (SSQ_K5P_FIRST=1) vs after the gather's (0): the riding-forward tests, bench.py's
# recon rates ABAB untraced, then one kernel-traced run each (recon HBM set, K14+K5p rows).
TAG=${1:-r5k5}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_recon_gpu.py -m gpu -q -x -k "prepared or rides or fused_matches or recon_fused" --timeout 120 --timeout-method thread > $OUT/pytest_$TAG.log 2>&1 || { echo "tests failed"; grep -E "FAILED|passed|failed" $OUT/pytest_$TAG.log | head; exit 1; }
tail -1 $OUT/pytest_$TAG.log
for rep in 1 2; do
for F in 1 0; do
  SSQ_K5P_FIRST=$F timeout -k 10 400 python bench.py --no-cpu-baseline --no-validate --recon-iters 300 > $OUT/bench_${TAG}_f${F}_$rep.log 2>&1 || { echo "bench failed"; tail -5 $OUT/bench_${TAG}_f${F}_$rep.log; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['recon']; print('first $F rep $rep', r['resnet18_all_blocks_iters_per_s'], r['iters_per_s'])" $OUT/bench_${TAG}_f${F}_$rep.log
done
done
cd /tmp && export TMPDIR=/tmp
for F in 1 0; do
  N=${TAG}_f$F
  SSQ_K5P_FIRST=$F timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d $OUT/prof_$N -o bench -- python3 $R/bench.py --no-cpu-baseline --no-validate --recon-iters 100 > $OUT/prof_bench_$N.log 2>&1 || { echo "rocprof bench failed"; tail -5 $OUT/prof_bench_$N.log; exit 1; }
  KT=$(find $OUT/prof_$N -name "*kernel_trace.csv" | head -1)
  python3 $R/tools/recon_roofline.py "$KT" $OUT/recon_roofline_$N.json > $OUT/recon_roofline_$N.txt 2>&1
  rm -f "$KT"
  echo "first $F"; head -1 $OUT/recon_roofline_$N.txt | cut -c300-420
  grep "K14\|^layer" $OUT/recon_roofline_$N.txt | tr -s ' ' | cut -c1-70
done
exit 0
