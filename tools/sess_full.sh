R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
TAG=${1:-full}
SSQ_PARITY_LOG=$OUT/parity_$TAG.jsonl timeout -k 10 600 python -u -m pytest tests -m gpu -q --maxfail 5 --timeout 120 --timeout-method thread > $OUT/pytest_gpu_$TAG.log 2>&1
rc=$?; tail -2 $OUT/pytest_gpu_$TAG.log
if [ $rc -ne 0 ]; then echo "pytest rc=$rc"; grep -E "FAILED|Error" $OUT/pytest_gpu_$TAG.log | head -20; exit 1; fi
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke_$TAG.log 2>&1 || { echo smoke failed; tail $OUT/smoke_$TAG.log; exit 1; }
tail -1 $OUT/smoke_$TAG.log
timeout -k 10 600 python bench.py > $OUT/bench_$TAG.log 2>&1 || { tail -20 $OUT/bench_$TAG.log; exit 1; }
tail -1 $OUT/bench_$TAG.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline_recon']['frac'], d['recon']['resnet18_all_blocks_iters_per_s'], d['validation']['images_per_s'])"
bash tools/dist_bench2.sh > $OUT/dist2_$TAG.log 2>&1 || { echo "dist2 failed"; tail -30 $OUT/dist2_$TAG.log; exit 1; }
grep '"metric"' $OUT/dist2_$TAG.log | tail -1 | cut -c1-400
