#!/bin/bash
# One GPU box session: GPU tests, smoke, bench, rocprofv3 kernel-trace summary.
# Usage (via gpurun): bash tools/gpu_session.sh [tag]
# Any abort / segfault / timeout ends the session before the next GPU step.
TAG=${1:-run}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
rm -f $OUT/parity_$TAG.jsonl
SSQ_PARITY_LOG=$OUT/parity_$TAG.jsonl timeout -k 10 600 python -u -m pytest tests -m gpu -q --maxfail 5 --timeout 120 --timeout-method thread > $OUT/pytest_gpu_$TAG.log 2>&1
rc=$?
echo "pytest rc=$rc" >> $OUT/pytest_gpu_$TAG.log
tail -3 $OUT/pytest_gpu_$TAG.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest ended abnormally ($rc); stopping"; exit $rc; fi
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke_$TAG.log 2>&1 || { echo "smoke failed"; tail -20 $OUT/smoke_$TAG.log; exit 1; }
tail -1 $OUT/smoke_$TAG.log
timeout -k 10 600 python bench.py > $OUT/bench_$TAG.log 2>&1 || { echo "bench failed"; tail -20 $OUT/bench_$TAG.log; exit 1; }
tail -1 $OUT/bench_$TAG.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$TAG -o bench -- python3 $R/bench.py --no-cpu-baseline --recon-iters 100 > $OUT/prof_bench_$TAG.log 2>&1 || { echo "rocprof failed"; tail -20 $OUT/prof_bench_$TAG.log; exit 1; }
KT=$(find $OUT/prof_$TAG -name "*kernel_trace.csv" | head -1)
[ -n "$KT" ] && python3 $R/tools/trace_iter.py "$KT" > $OUT/iter_anatomy_$TAG.txt 2>&1
# the full trace is tens of MB (gpurun copies back <= 64 MiB): keep the summaries only
[ -n "$KT" ] && rm -f "$KT"
find $OUT/prof_$TAG -name "*stats*"
exit 0
