#!/bin/bash
# BRECQ act-phase conv cache: loop tests, the act-phase anatomy and the end-to-end time.
TAG=${1:-ac}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
timeout -k 10 300 python -u -m pytest tests/test_recon_gpu.py tests/test_recon2_gpu.py tests/test_dp_gpu.py -m gpu -q -k "brecq or knobs or layer_recon or act" --timeout 120 --timeout-method thread > $OUT/pytest_$TAG.log 2>&1
rc=$?
tail -3 $OUT/pytest_$TAG.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest abnormal $rc"; exit $rc; fi
bash tools/act_anatomy.sh $TAG || exit 1
cd $R
timeout -k 10 600 python main_imagenet.py --arch resnet18 --n_bits_w 2 --n_bits_a 4 --weight 1.0 --bias_cal True --bias_ch_quant True > $OUT/e2e_$TAG.log 2>&1 || { echo "e2e failed"; tail -20 $OUT/e2e_$TAG.log; exit 1; }
grep "calibration finished" $OUT/e2e_$TAG.log | cut -c1-160
