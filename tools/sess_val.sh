# f3 validation: rocprofv3 kernel trace of the validation bench, per-batch breakdown
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
TAG=${1:-val}
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/val_$TAG -o val -- python3 $R/tools/val_profile.py > $OUT/val_$TAG.log 2>&1 || { echo "val profile failed"; tail $OUT/val_$TAG.log; exit 1; }
grep '"metric"' $OUT/val_$TAG.log
KT=$(find $OUT/val_$TAG -name "*kernel_trace.csv" | head -1)
python3 $R/tools/val_summary.py "$KT" 20 > $OUT/val_sum_$TAG.txt 2>&1; rm -f "$KT"; cat $OUT/val_sum_$TAG.txt
