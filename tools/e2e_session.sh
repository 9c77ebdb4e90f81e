#!/bin/bash
# End-to-end calibration runs of the README entry point on one GPU (synthetic data):
# resnet18 W2A4 shifted-scale (bias_cal + bias_ch_quant), resnet50 / mobilenetv2 W2A4 BRECQ.
TAG=${1:-run}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
timeout -k 10 600 python main_imagenet.py --arch resnet18 --n_bits_w 2 --n_bits_a 4 --bias_cal True --bias_ch_quant True --num_samples 256 --shift_iters 100 --iters_w 100 --iters_a 100 > $OUT/e2e_r18_$TAG.log 2>&1 || { echo "resnet18 failed"; tail -30 $OUT/e2e_r18_$TAG.log; exit 1; }
tail -2 $OUT/e2e_r18_$TAG.log
timeout -k 10 600 python main_imagenet.py --arch resnet50 --n_bits_w 2 --n_bits_a 4 --num_samples 128 --iters_w 50 --iters_a 50 > $OUT/e2e_r50_$TAG.log 2>&1 || { echo "resnet50 failed"; tail -30 $OUT/e2e_r50_$TAG.log; exit 1; }
tail -2 $OUT/e2e_r50_$TAG.log
timeout -k 10 600 python main_imagenet.py --arch regnetx_3200m --n_bits_w 2 --n_bits_a 4 --bias_ch_quant True --num_samples 128 --shift_iters 50 --iters_w 50 --iters_a 50 > $OUT/e2e_rgx_$TAG.log 2>&1 || { echo "regnetx failed"; tail -30 $OUT/e2e_rgx_$TAG.log; exit 1; }
tail -2 $OUT/e2e_rgx_$TAG.log
timeout -k 10 600 python main_imagenet.py --arch mobilenetv2 --n_bits_w 2 --n_bits_a 4 --bias_ch_quant True --num_samples 128 --shift_iters 50 --iters_w 50 --iters_a 50 > $OUT/e2e_mbv2_$TAG.log 2>&1 || { echo "mobilenetv2 failed"; tail -30 $OUT/e2e_mbv2_$TAG.log; exit 1; }
tail -2 $OUT/e2e_mbv2_$TAG.log
