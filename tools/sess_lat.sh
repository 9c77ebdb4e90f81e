# kernel-duration floor probe (tools/latency_probe.hip) under rocprofv3 --kernel-trace
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
TAG=${1:-lat}
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $OUT/lat_$TAG -o lat -- $R/tools/latency_probe > $OUT/lat_$TAG.log 2>&1 || { echo "latency probe failed"; tail $OUT/lat_$TAG.log; exit 1; }
KT=$(find $OUT/lat_$TAG -name "*kernel_trace.csv" | head -1)
python3 $R/tools/latency_summary.py "$KT" > $OUT/lat_sum_$TAG.txt 2>&1; cat $OUT/lat_sum_$TAG.txt
