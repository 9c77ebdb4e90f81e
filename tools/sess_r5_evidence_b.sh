#!/bin/bash
# Round-end evidence, part B: the end-to-end calibration (profiled kernel stats, unprofiled
# wall time, per-call breakdown), the act phase's and the fc loop's iteration anatomy, the
# short runs of the other model families, and bench.py --gpus 2 self-launched over gloo.
TAG=${1:-r5e}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
A="--arch resnet18 --n_bits_w 2 --n_bits_a 4 --weight 1.0 --bias_cal True --bias_ch_quant True"
timeout -k 10 600 python main_imagenet.py $A > $OUT/e2e_$TAG.log 2>&1 || { echo "e2e failed"; tail -20 $OUT/e2e_$TAG.log; exit 1; }
grep "calibration finished" $OUT/e2e_$TAG.log | cut -c1-160
SSQ_BREAKDOWN_HOOK=0 timeout -k 10 300 python tools/e2e_breakdown.py $A > $OUT/bd_$TAG.log 2>&1 || { echo "breakdown failed"; tail -5 $OUT/bd_$TAG.log; exit 1; }
grep "^\[breakdown\] \(total\|[a-z_]* *[0-9]* calls\)" $OUT/bd_$TAG.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/e2eprof -o e2e -- python3 $R/main_imagenet.py $A > $OUT/e2e_prof_$TAG.log 2>&1 || { echo "e2e profiled failed"; tail -20 $OUT/e2e_prof_$TAG.log; exit 1; }
cp $(find /tmp/e2eprof -name "*kernel_stats.csv" | head -1) $OUT/e2e_kernel_stats_$TAG.csv
rm -rf /tmp/e2eprof
grep "calibration finished" $OUT/e2e_prof_$TAG.log | cut -c1-160
cd $R
bash tools/act_anatomy.sh $TAG || exit 1
SSQ_FUSE_FC=1 SSQ_BRECQ_CHUNK=25 timeout -k 10 300 python tools/fc_recon_rate.py > $OUT/fc_rate_$TAG.log 2>&1 || { echo "fc rate failed"; exit 1; }
grep fc_adaround $OUT/fc_rate_$TAG.log
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $OUT/prof_fc_$TAG -o fc -- python3 $R/tools/fc_recon_rate.py > $OUT/prof_fc_$TAG.log 2>&1 || { echo "rocprof fc failed"; exit 1; }
KT=$(find $OUT/prof_fc_$TAG -name "*kernel_trace.csv" | head -1)
MARKER=fc_fwd_loss python3 $R/tools/trace_iter.py "$KT" > $OUT/fc_anatomy_$TAG.txt 2>&1
rm -f "$KT"
cd $R
bash tools/e2e_session.sh $TAG || exit 1
timeout -k 10 400 python bench.py --gpus 2 --dist-backend gloo --steps 20 --warmup 5 --no-cpu-baseline --recon-iters 30 > $OUT/dist2_$TAG.log 2>&1 || { echo "dist2 failed"; tail -20 $OUT/dist2_$TAG.log; exit 1; }
tail -1 $OUT/dist2_$TAG.log | cut -c1-200
exit 0
