# prepared adaShift kernels: parity tests, then cold-cache launch durations per block
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
TAG=${1:-al}
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "prepared or adashift or armed" -m gpu -q -x --timeout 120 --timeout-method thread > $OUT/pytest_$TAG.log 2>&1 || { tail -20 $OUT/pytest_$TAG.log; exit 1; }
tail -1 $OUT/pytest_$TAG.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $OUT/cold_$TAG -o cold -- python3 $R/tools/alpha_cold.py 40 > $OUT/cold_$TAG.log 2>&1 || { echo "cold failed"; tail $OUT/cold_$TAG.log; exit 1; }
KT=$(find $OUT/cold_$TAG -name "*kernel_trace.csv" | head -1)
python3 $R/tools/trace_avg.py "$KT" shift_fwd_prep alpha_bwd_prep --groups=5 > $OUT/cold_avg_$TAG.txt; rm -f "$KT"
cat $OUT/cold_avg_$TAG.txt
