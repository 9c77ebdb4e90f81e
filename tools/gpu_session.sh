#!/bin/bash
# One GPU box session: GPU tests, smoke, bench, rocprofv3 kernel-trace summary.
# Usage (via gpurun): bash tools/gpu_session.sh [tag]
TAG=${1:-run}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
timeout -k 10 600 python -m pytest tests -m gpu -q > $OUT/pytest_gpu_$TAG.log 2>&1
echo "pytest rc=$?" >> $OUT/pytest_gpu_$TAG.log
tail -3 $OUT/pytest_gpu_$TAG.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke_$TAG.log 2>&1 || { echo "smoke failed"; tail -20 $OUT/smoke_$TAG.log; exit 1; }
tail -1 $OUT/smoke_$TAG.log
timeout -k 10 600 python bench.py > $OUT/bench_$TAG.log 2>&1 || { echo "bench failed"; tail -20 $OUT/bench_$TAG.log; exit 1; }
tail -1 $OUT/bench_$TAG.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$TAG -o bench -- python3 $R/bench.py --no-cpu-baseline --recon-iters 100 > $OUT/prof_bench_$TAG.log 2>&1 || { echo "rocprof failed"; tail -20 $OUT/prof_bench_$TAG.log; exit 1; }
find $OUT/prof_$TAG -name "*stats*" | head
