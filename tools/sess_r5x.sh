#!/bin/bash
# r5x A/B: K6p's per-channel form with the XCD-aware channel order (SSQ_K6P_XCD) on / off,
# at r4's reach (Co*K <= 1280, 1x1 Co <= 128) and extended to every ResNet-18 conv
# (Co*K <= 5120; 1x1 Co <= 4096): cold whole-block launches (tools/alpha_cold.py).
TAG=${1:-r5x}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for X in 0 1; do
for V in "1280 128" "5120 128" "5120 4096"; do
  set -- $V
  N=k6p_${TAG}_x${X}_$1_$2
  SSQ_K6P_XCD=$X SSQ_K6P_CHAN_ELEMS=$1 SSQ_K6P_CHAN_CO=$2 timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $OUT/$N -o t -- python3 $R/tools/alpha_cold.py 30 > $OUT/$N.log 2>&1 || { echo "alpha_cold $X $V failed"; tail -5 $OUT/$N.log; exit 1; }
  KT=$(find $OUT/$N -name "*kernel_trace.csv" | head -1)
  python3 $R/tools/trace_avg.py "$KT" alpha_bwd --groups=5 > $OUT/$N.txt 2>&1
  rm -f "$KT"
  echo "## XCD=$X ELEMS/CO=$V"; cat $OUT/$N.txt | cut -c1-60
done
done
exit 0
