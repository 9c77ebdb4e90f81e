#!/bin/bash
# r5b A/B: the fc AdaRound loop with one vs 25 iterations per graph replay (rate + anatomy),
# and K6p's per-channel form extended to Co*K <= 5120 (cold-cache launches + in-loop trace).
TAG=${1:-r5b}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
for C in 1 25; do
  SSQ_BRECQ_CHUNK=$C timeout -k 10 300 python tools/fc_recon_rate.py > $OUT/fc_rate_${TAG}_c$C.log 2>&1 || { echo "fc rate $C failed"; tail -5 $OUT/fc_rate_${TAG}_c$C.log; exit 1; }
  head -1 $OUT/fc_rate_${TAG}_c$C.log
done
cd /tmp && export TMPDIR=/tmp
for C in 1 25; do
  SSQ_BRECQ_CHUNK=$C timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $OUT/prof_fc_${TAG}_c$C -o fc -- python3 $R/tools/fc_recon_rate.py > $OUT/prof_fc_${TAG}_c$C.log 2>&1 || { echo "rocprof fc failed"; exit 1; }
  KT=$(find $OUT/prof_fc_${TAG}_c$C -name "*kernel_trace.csv" | head -1)
  python3 $R/tools/trace_iter.py "$KT" > $OUT/fc_anatomy_${TAG}_c$C.txt 2>&1
  rm -f "$KT"
  grep -- "---" $OUT/fc_anatomy_${TAG}_c$C.txt | tail -2
done
for V in "1280 128" "5120 128" "5120 4096"; do
  set -- $V
  SSQ_K6P_CHAN_ELEMS=$1 SSQ_K6P_CHAN_CO=$2 timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $OUT/k6p_${TAG}_$1_$2 -o t -- python3 $R/tools/alpha_cold.py 30 > $OUT/k6p_${TAG}_$1_$2.log 2>&1 || { echo "alpha_cold $V failed"; exit 1; }
  KT=$(find $OUT/k6p_${TAG}_$1_$2 -name "*kernel_trace.csv" | head -1)
  python3 $R/tools/trace_avg.py "$KT" alpha_bwd --groups=5 > $OUT/k6p_${TAG}_$1_$2.txt 2>&1
  rm -f "$KT"
done
for V in 1280 5120; do
  SSQ_K6P_CHAN_ELEMS=$V timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d $OUT/prof_${TAG}_$V -o bench -- python3 $R/bench.py --no-cpu-baseline --no-validate --recon-iters 100 > $OUT/prof_bench_${TAG}_$V.log 2>&1 || { echo "rocprof bench $V failed"; tail -5 $OUT/prof_bench_${TAG}_$V.log; exit 1; }
  KT=$(find $OUT/prof_${TAG}_$V -name "*kernel_trace.csv" | head -1)
  python3 $R/tools/recon_roofline.py "$KT" $OUT/recon_roofline_${TAG}_$V.json > $OUT/recon_roofline_${TAG}_$V.txt 2>&1
  rm -f "$KT"
  head -1 $OUT/recon_roofline_${TAG}_$V.txt | cut -c1-400
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('$V', d['recon']['resnet18_all_blocks_iters_per_s'], d['recon']['iters_per_s'])" $OUT/prof_bench_${TAG}_$V.log
done
exit 0
