#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for V in "1536 8" "768 8" "3072 8" "1536 16" "768 16" "3072 4"; do
  set -- $V
  SSQ_PREP_WGS=$1 SSQ_PREP_ROWS=$2 timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $OUT/k6pab_$1_$2 -o t -- python3 $R/tools/alpha_cold.py 30 > $OUT/k6pab_$1_$2.log 2>&1 || { echo "ab $V failed"; tail -5 $OUT/k6pab_$1_$2.log; exit 1; }
  KT=$(find $OUT/k6pab_$1_$2 -name "*kernel_trace.csv" | head -1)
  python3 $R/tools/trace_avg.py "$KT" alpha_bwd --groups=5 > $OUT/k6pab_$1_$2.txt 2>&1
  python3 $R/tools/trace_avg.py "$KT" shift_fwd --groups=5 > $OUT/k5pab_$1_$2.txt 2>&1
  rm -f "$KT"
  echo "== WGS=$1 ROWS=$2"; cat $OUT/k6pab_$1_$2.txt | cut -c1-60; cat $OUT/k5pab_$1_$2.txt | cut -c1-60
done
