#!/bin/bash
# r5c: the two tests fixed after r5a, the launch-floor probe, then the r5b A/Bs.
TAG=${1:-r5c}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
bash tools/sess_tests.sh $TAG "frozen_loop or real_layer_shift or chunked or into_gemm or fused_epilogue"
rc=$?
[ $rc -gt 1 ] && exit $rc
timeout -k 10 120 ./tools/floor_probe > $OUT/floor_probe_$TAG.json 2>&1 || { echo "floor probe failed"; tail -5 $OUT/floor_probe_$TAG.json; exit 1; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $OUT/floorprof_$TAG -o fp -- $R/tools/floor_probe > $OUT/floor_probe_prof_$TAG.json 2>&1 || { echo "rocprof floor probe failed"; exit 1; }
KT=$(find $OUT/floorprof_$TAG -name "*kernel_trace.csv" | head -1)
python3 $R/tools/floor_summary.py "$KT" > $OUT/floor_trace_$TAG.txt 2>&1
cp "$KT" $OUT/floor_trace_$TAG.csv
rm -f "$KT"
cd $R
bash tools/sess_r5b.sh $TAG
