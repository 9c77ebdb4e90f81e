R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
TAG=${1:-gemm}
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -q -x --timeout 120 --timeout-method thread -k "wgrad" > $OUT/pytest_$TAG.log 2>&1 || { tail -30 $OUT/pytest_$TAG.log; exit 1; }
tail -2 $OUT/pytest_$TAG.log
SSQ_PARITY_LOG=$OUT/parity_$TAG.jsonl timeout -k 10 600 python -u -m pytest tests -m gpu -q --maxfail 5 --timeout 120 --timeout-method thread > $OUT/pytest_gpu_$TAG.log 2>&1
rc=$?; tail -2 $OUT/pytest_gpu_$TAG.log
if [ $rc -ne 0 ]; then echo "pytest rc=$rc"; grep -E "FAILED|Error|error" $OUT/pytest_gpu_$TAG.log | head -30; exit 1; fi
timeout -k 10 600 python bench.py --no-cpu-baseline --no-validate > $OUT/bench_$TAG.log 2>&1 || { tail -20 $OUT/bench_$TAG.log; exit 1; }
tail -1 $OUT/bench_$TAG.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['roofline']['frac'], d['roofline_recon']['frac'], d['recon']['resnet18_all_blocks_iters_per_s'], d['recon']['resnet18_all_blocks_iters_per_s_benchmark_solvers'], d['recon']['iters_per_s'])"
