#!/bin/bash
# GPU suite, then the full ResNet-18 W2A4 --bias_cal flow under tools/e2e_breakdown.py: one
# process to warm the box, one with per-call times, one with the per-iteration hook (setup /
# warm-up / capture / steady phases of every BRECQ loop).
TAG=${1:-r5v}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
SSQ_PARITY_LOG=$OUT/parity_$TAG.jsonl timeout -k 10 500 python -u -m pytest tests -m gpu -q --maxfail 10 --timeout 120 --timeout-method thread > $OUT/pytest_$TAG.log 2>&1
rc=$?
tail -2 $OUT/pytest_$TAG.log
[ $rc -ne 0 ] && { echo "pytest rc=$rc"; grep -E "^(FAILED|ERROR)" $OUT/pytest_$TAG.log | head; exit $rc; }
A="--arch resnet18 --n_bits_w 2 --n_bits_a 4 --weight 1.0 --bias_cal True --bias_ch_quant True"
for V in cold warm; do
  SSQ_BREAKDOWN_HOOK=0 timeout -k 10 300 python tools/e2e_breakdown.py $A > $OUT/bd_${TAG}_$V.log 2>&1 || { echo "breakdown $V failed"; tail -5 $OUT/bd_${TAG}_$V.log; exit 1; }
  echo "== $V"; grep "calibration finished\|brecq_loop #\|\[breakdown\] total" $OUT/bd_${TAG}_$V.log | cut -c1-150
done
SSQ_BREAKDOWN_HOOK=1 timeout -k 10 300 python tools/e2e_breakdown.py $A > $OUT/bd_${TAG}_hook.log 2>&1 || { echo "breakdown hook failed"; tail -5 $OUT/bd_${TAG}_hook.log; exit 1; }
echo "== hook"; grep "calibration finished\|brecq setup" $OUT/bd_${TAG}_hook.log | cut -c1-200
exit 0
