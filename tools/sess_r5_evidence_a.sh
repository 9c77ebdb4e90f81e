#!/bin/bash
# Round-end evidence, part A, at the tree's kernels: GPU suite + smoke, the bench line, a
# rocprofv3 kernel trace of the bench (K1 launch stats, the recon roofline JSON, the iteration
# anatomy), the two PMC passes (HBM traffic JSON).
# Usage (via gpurun): SSQ_GIT_SHA=<sha> bash tools/sess_r5_evidence_a.sh TAG
TAG=${1:-r5e}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
SSQ_PARITY_LOG=$OUT/parity_$TAG.jsonl timeout -k 10 500 python -u -m pytest tests -m gpu -q --maxfail 10 --timeout 120 --timeout-method thread > $OUT/pytest_$TAG.log 2>&1
rc=$?
echo "pytest rc=$rc" >> $OUT/pytest_$TAG.log
tail -2 $OUT/pytest_$TAG.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest ended abnormally ($rc)"; exit $rc; fi
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke_$TAG.log 2>&1 || { echo "smoke failed"; tail -20 $OUT/smoke_$TAG.log; exit 1; }
tail -1 $OUT/smoke_$TAG.log
timeout -k 10 600 python bench.py > $OUT/bench_$TAG.log 2>&1 || { echo "bench failed"; tail -20 $OUT/bench_$TAG.log; exit 1; }
tail -1 $OUT/bench_$TAG.log | cut -c1-300
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$TAG -o bench -- python3 $R/bench.py --no-cpu-baseline --no-validate --recon-iters 100 > $OUT/prof_bench_$TAG.log 2>&1 || { echo "rocprof failed"; tail -20 $OUT/prof_bench_$TAG.log; exit 1; }
KT=$(find $OUT/prof_$TAG -name "*kernel_trace.csv" | head -1)
python3 $R/tools/k1_trace_stats.py "$KT" > $OUT/k1_trace_$TAG.json 2>&1
python3 $R/tools/recon_roofline.py "$KT" $OUT/recon_roofline_$TAG.json > $OUT/recon_roofline_$TAG.txt 2>&1
python3 $R/tools/trace_iter.py "$KT" > $OUT/iter_anatomy_$TAG.txt 2>&1
rm -f "$KT"
head -1 $OUT/recon_roofline_$TAG.txt | cut -c1-300
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch_$TAG -o f -- python3 $R/bench.py --no-recon --no-validate --no-cpu-baseline --steps 3 --warmup 1 > $OUT/pmc_fetch_$TAG.log 2>&1 || { echo "fetch pass failed"; tail -20 $OUT/pmc_fetch_$TAG.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write_$TAG -o w -- python3 $R/bench.py --no-recon --no-validate --no-cpu-baseline --steps 3 --warmup 1 > $OUT/pmc_write_$TAG.log 2>&1 || { echo "write pass failed"; tail -20 $OUT/pmc_write_$TAG.log; exit 1; }
python3 $R/tools/pmc_traffic.py $OUT/pmc_fetch_$TAG $OUT/pmc_write_$TAG $OUT/pmc_traffic_$TAG.json > /dev/null 2>&1
find $OUT/pmc_fetch_$TAG $OUT/pmc_write_$TAG -name "*counter_collection.csv" -delete
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print({k: v.get('hbm_bytes_per_launch') for k, v in d.items() if isinstance(v, dict) and 'hbm_bytes_per_launch' in v})" $OUT/pmc_traffic_$TAG.json
exit 0
