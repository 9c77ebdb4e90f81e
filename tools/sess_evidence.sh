# Round evidence: GPU tests, smoke, the default bench line, a rocprofv3 kernel-trace --stats
# pass of the same bench (+ recon iteration anatomy), the world-2 gloo bench rehearsal.
# SKIP_TESTS=1 skips pytest + smoke, SKIP_DIST=1 the world-2 rehearsal.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
TAG=${1:-ev}
if [ -z "$SKIP_TESTS" ]; then
SSQ_PARITY_LOG=$OUT/parity_$TAG.jsonl timeout -k 10 600 python -u -m pytest tests -m gpu -q --maxfail 5 --timeout 120 --timeout-method thread > $OUT/pytest_gpu_$TAG.log 2>&1
rc=$?; tail -2 $OUT/pytest_gpu_$TAG.log
if [ $rc -ne 0 ]; then echo "pytest rc=$rc"; grep -E "FAILED|Error|error" $OUT/pytest_gpu_$TAG.log | head -30; exit 1; fi
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke_$TAG.log 2>&1 || { echo smoke failed; tail $OUT/smoke_$TAG.log; exit 1; }
tail -1 $OUT/smoke_$TAG.log
fi
timeout -k 10 600 python bench.py > $OUT/bench_$TAG.log 2>&1 || { tail -20 $OUT/bench_$TAG.log; exit 1; }
tail -1 $OUT/bench_$TAG.log | cut -c1-300
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$TAG -o bench -- python3 $R/bench.py --no-cpu-baseline --recon-iters 100 > $OUT/prof_bench_$TAG.log 2>&1 || { echo "rocprof failed"; tail -20 $OUT/prof_bench_$TAG.log; exit 1; }
KT=$(find $OUT/prof_$TAG -name "*kernel_trace.csv" | head -1)
[ -n "$KT" ] && python3 $R/tools/trace_iter.py "$KT" > $OUT/iter_anatomy_$TAG.txt 2>&1
# the headline kernel's full-size launches only (the stats average also holds small ones)
[ -n "$KT" ] && python3 $R/tools/k1_trace_stats.py "$KT" > $OUT/k1_trace_$TAG.json 2>&1
# the recon roofline priced on the loop's own launches (bench.py reports profiles/recon_roofline.json)
[ -n "$KT" ] && python3 $R/tools/recon_roofline.py "$KT" $OUT/recon_roofline_$TAG.json > $OUT/recon_roofline_$TAG.txt 2>&1
[ -n "$KT" ] && rm -f "$KT"
cd $R
[ -n "$SKIP_DIST" ] && exit 0
bash tools/dist_bench2.sh > $OUT/dist2_$TAG.log 2>&1 || { echo "dist2 failed"; tail -30 $OUT/dist2_$TAG.log; exit 1; }
grep '"metric"' $OUT/dist2_$TAG.log | tail -1 | cut -c1-200
