R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
timeout -k 10 300 python -u -m pytest tests/test_recon2_gpu.py tests/test_dp_gpu.py -q -x --timeout 120 --timeout-method thread -k "validation" > $OUT/f3_tests.log 2>&1 || { tail -30 $OUT/f3_tests.log; exit 1; }
tail -3 $OUT/f3_tests.log
grep PARITY $OUT/f3_tests.log || true
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $OUT/anat_l1 -o t -- python3 $R/tools/block_anatomy.py resnet18 layer1.0 60 1 256 > $OUT/anat_l1.log 2>&1 || { tail $OUT/anat_l1.log; exit 1; }
KT=$(find $OUT/anat_l1 -name "*kernel_trace.csv" | head -1)
python3 $R/tools/trace_iter.py "$KT" full > $OUT/anat_l1_full.txt 2>&1
rm -f "$KT"
cd $R
timeout -k 10 600 python bench.py --no-cpu-baseline --recon-iters 50 > $OUT/bench_f3.log 2>&1 || { tail -20 $OUT/bench_f3.log; exit 1; }
tail -1 $OUT/bench_f3.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['validation'])"
