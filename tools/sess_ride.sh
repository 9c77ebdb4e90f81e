# r3: the bench step as one launch -- kernel test, bench line, PMC traffic of the step kernel,
# rocprofv3 trace stats of the step kernel
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
TAG=${1:-ride}
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "ride or multi or fq" -m gpu -q -x --timeout 120 --timeout-method thread > $OUT/pytest_$TAG.log 2>&1 || { tail -30 $OUT/pytest_$TAG.log; exit 1; }
tail -1 $OUT/pytest_$TAG.log
timeout -k 10 300 python bench.py --no-recon --no-validate --no-cpu-baseline > $OUT/bench_$TAG.log 2>&1 || { tail -20 $OUT/bench_$TAG.log; exit 1; }
tail -1 $OUT/bench_$TAG.log | cut -c1-400
bash tools/pmc_session.sh $TAG > $OUT/pmc_$TAG.log 2>&1 || { tail -20 $OUT/pmc_$TAG.log; exit 1; }
cat $OUT/pmc_traffic_$TAG.json | head -30
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$TAG -o bench -- python3 $R/bench.py --no-recon --no-validate --no-cpu-baseline > $OUT/prof_bench_$TAG.log 2>&1 || { echo "rocprof failed"; tail -20 $OUT/prof_bench_$TAG.log; exit 1; }
KT=$(find $OUT/prof_$TAG -name "*kernel_trace.csv" | head -1)
python3 $R/tools/k1_trace_stats.py "$KT" > $OUT/k1_trace_$TAG.json; rm -f "$KT"; cat $OUT/k1_trace_$TAG.json
