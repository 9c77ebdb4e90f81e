# r3: the wave-column alpha backward / hoisted K5p -- parity tests first, then cold-cache
# launch durations (one- vs two-launch), the kernel-duration floor probe, hot graph timing.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
TAG=${1:-al}
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -k "prepared or adashift" -m gpu -q -x --timeout 120 --timeout-method thread > $OUT/pytest_$TAG.log 2>&1
rc=$?; tail -3 $OUT/pytest_$TAG.log
if [ $rc -ne 0 ]; then grep -E "FAILED|Error|assert" $OUT/pytest_$TAG.log | head -30; exit 1; fi
cd /tmp && export TMPDIR=/tmp
for two in 0 1 2; do
  SSQ_ALPHA_ONE_LAUNCH=$([ $two = 1 ] && echo 1 || echo 0) SSQ_PREP_BWD_LEGACY=$([ $two = 2 ] && echo 1 || echo 0) timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $OUT/cold_$TAG$two -o cold -- python3 $R/tools/alpha_cold.py 40 > $OUT/cold_$TAG$two.log 2>&1 || { echo "cold $two failed"; tail $OUT/cold_$TAG$two.log; exit 1; }
  KT=$(find $OUT/cold_$TAG$two -name "*kernel_trace.csv" | head -1)
  python3 $R/tools/trace_avg.py "$KT" shift_fwd_prep alpha_bwd --groups=5 > $OUT/cold_avg_$TAG$two.txt; rm -f "$KT"
  echo "variant=$two (0 wave-column + stage 2, 1 wave-column one launch, 2 legacy thread-column + stage 2)"; cat $OUT/cold_avg_$TAG$two.txt
done
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $OUT/lat_$TAG -o lat -- $R/tools/latency_probe > $OUT/lat_$TAG.log 2>&1 || { echo "latency probe failed"; tail $OUT/lat_$TAG.log; exit 1; }
KT=$(find $OUT/lat_$TAG -name "*kernel_trace.csv" | head -1)
python3 $R/tools/latency_summary.py "$KT" > $OUT/lat_sum_$TAG.txt; rm -f "$KT"; cat $OUT/lat_sum_$TAG.txt
cd $R
timeout -k 10 120 python -u tools/adashift_bench.py --blocks > $OUT/ada_hot_$TAG.log 2>&1; tail -1 $OUT/ada_hot_$TAG.log
