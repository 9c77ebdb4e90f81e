#!/bin/bash
# r5d: the new / changed tests, then the fc loop: unfused vs K19 fused, 1 vs 25 iterations
# per graph replay (rates unprofiled; anatomy of the fused chunked loop under rocprofv3).
TAG=${1:-r5d}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
bash tools/sess_tests.sh $TAG "${2:-into_gemm or fc_ or chunked or frozen_loop or real_layer_shift or layer_reconstruction}"
rc=$?
[ $rc -gt 1 ] && exit $rc
for V in "0 25" "1 1" "1 25"; do
  set -- $V
  SSQ_FUSE_FC=$1 SSQ_BRECQ_CHUNK=$2 timeout -k 10 300 python tools/fc_recon_rate.py > $OUT/fc_rate_${TAG}_f$1_c$2.log 2>&1 || { echo "fc rate $V failed"; tail -5 $OUT/fc_rate_${TAG}_f$1_c$2.log; exit 1; }
  echo "fuse=$1 chunk=$2 $(grep fc_adaround $OUT/fc_rate_${TAG}_f$1_c$2.log)"
done
cd /tmp && export TMPDIR=/tmp
SSQ_FUSE_FC=1 SSQ_BRECQ_CHUNK=25 timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $OUT/prof_fc_$TAG -o fc -- python3 $R/tools/fc_recon_rate.py > $OUT/prof_fc_$TAG.log 2>&1 || { echo "rocprof fc failed"; exit 1; }
KT=$(find $OUT/prof_fc_$TAG -name "*kernel_trace.csv" | head -1)
MARKER=fc_fwd_loss python3 $R/tools/trace_iter.py "$KT" > $OUT/fc_anatomy_$TAG.txt 2>&1
rm -f "$KT"
grep -- "---" $OUT/fc_anatomy_$TAG.txt | tail -2
exit $rc
