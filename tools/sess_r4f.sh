#!/bin/bash
# GPU suite, the act-phase anatomy trace and an unprofiled end-to-end W2A4 calibration run.
TAG=${1:-r4f}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
SSQ_PARITY_LOG=$OUT/parity_$TAG.jsonl timeout -k 10 500 python -u -m pytest tests -m gpu -q --maxfail 10 --timeout 120 --timeout-method thread > $OUT/pytest_$TAG.log 2>&1
rc=$?
echo "pytest rc=$rc" >> $OUT/pytest_$TAG.log
tail -2 $OUT/pytest_$TAG.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest ended abnormally ($rc)"; exit $rc; fi
bash tools/act_anatomy.sh $TAG || exit 1
cd $R
timeout -k 10 600 python main_imagenet.py --arch resnet18 --n_bits_w 2 --n_bits_a 4 --weight 1.0 --bias_cal True --bias_ch_quant True > $OUT/e2e_$TAG.log 2>&1 || { echo "e2e failed"; tail -20 $OUT/e2e_$TAG.log; exit 1; }
grep "calibration finished" $OUT/e2e_$TAG.log | cut -c1-160
