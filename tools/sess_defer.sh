R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
TAG=${1:-defer}
SSQ_PARITY_LOG=$OUT/parity_$TAG.jsonl timeout -k 10 600 python -u -m pytest tests -m gpu -q --maxfail 5 --timeout 120 --timeout-method thread > $OUT/pytest_gpu_$TAG.log 2>&1
rc=$?; tail -2 $OUT/pytest_gpu_$TAG.log
if [ $rc -ne 0 ]; then echo "pytest rc=$rc"; grep -E "FAILED|Error|error" $OUT/pytest_gpu_$TAG.log | head -30; exit 1; fi
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $OUT/anat_$TAG -o t -- python3 $R/tools/block_anatomy.py resnet18 layer1.0 60 1 256 > $OUT/anat_$TAG.log 2>&1 || { tail $OUT/anat_$TAG.log; exit 1; }
KT=$(find $OUT/anat_$TAG -name "*kernel_trace.csv" | head -1)
python3 $R/tools/trace_iter.py "$KT" full > $OUT/anat_${TAG}_full.txt 2>&1
rm -f "$KT"
head -22 $OUT/anat_${TAG}_full.txt | cut -c1-150
cd $R
timeout -k 10 600 python bench.py --no-cpu-baseline --no-validate > $OUT/bench_$TAG.log 2>&1 || { tail -20 $OUT/bench_$TAG.log; exit 1; }
tail -1 $OUT/bench_$TAG.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['roofline']['frac'], d['roofline_recon']['frac'], d['recon']['resnet18_all_blocks_iters_per_s'], d['recon']['iters_per_s'])"
