#!/bin/bash
# r5y A/B in the loop: K6p per-channel reach (SSQ_K6P_CHAN_ELEMS / SSQ_K6P_CHAN_CO) and the
# XCD-aware channel order (SSQ_K6P_XCD): bench.py's recon rates, ABAB untraced, then one
# kernel-traced run per variant for the recon HBM set (tools/recon_roofline.py).
TAG=${1:-r5y}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
VARS=("1 1280 128" "1 2304 256" "0 1280 128")
for rep in 1 2; do
for V in "${VARS[@]}"; do
  set -- $V
  N=${TAG}_x$1_$2_$3_$rep
  SSQ_K6P_XCD=$1 SSQ_K6P_CHAN_ELEMS=$2 SSQ_K6P_CHAN_CO=$3 timeout -k 10 400 python bench.py --no-cpu-baseline --no-validate --recon-iters 300 > $OUT/bench_$N.log 2>&1 || { echo "bench $V failed"; tail -5 $OUT/bench_$N.log; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['recon']; print('$V rep $rep', r['resnet18_all_blocks_iters_per_s'], r['iters_per_s'])" $OUT/bench_$N.log
done
done
cd /tmp && export TMPDIR=/tmp
for V in "${VARS[@]}"; do
  set -- $V
  N=${TAG}_x$1_$2_$3
  SSQ_K6P_XCD=$1 SSQ_K6P_CHAN_ELEMS=$2 SSQ_K6P_CHAN_CO=$3 timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d $OUT/prof_$N -o bench -- python3 $R/bench.py --no-cpu-baseline --no-validate --recon-iters 100 > $OUT/prof_bench_$N.log 2>&1 || { echo "rocprof bench $V failed"; tail -5 $OUT/prof_bench_$N.log; exit 1; }
  KT=$(find $OUT/prof_$N -name "*kernel_trace.csv" | head -1)
  python3 $R/tools/recon_roofline.py "$KT" $OUT/recon_roofline_$N.json > $OUT/recon_roofline_$N.txt 2>&1
  rm -f "$KT"
  echo "$V"; head -1 $OUT/recon_roofline_$N.txt | cut -c300-420
  grep "K6p\|^layer" $OUT/recon_roofline_$N.txt
done
exit 0
