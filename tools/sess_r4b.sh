#!/bin/bash
# r4 session: the GPU suite, the K6p alpha-backward forms A/B (tools/alpha_cold.py under
# rocprofv3, per block) and the recon rate per form.  Usage (via gpurun): bash tools/sess_r4b.sh TAG
TAG=${1:-r4b}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
SSQ_PARITY_LOG=$OUT/parity_$TAG.jsonl timeout -k 10 500 python -u -m pytest tests -m gpu -q --maxfail 10 --timeout 120 --timeout-method thread > $OUT/pytest_$TAG.log 2>&1
rc=$?
echo "pytest rc=$rc" >> $OUT/pytest_$TAG.log
tail -3 $OUT/pytest_$TAG.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest ended abnormally ($rc)"; exit $rc; fi
SSQ_K6P_FORM=2 timeout -k 10 200 python -u -m pytest tests/test_kernels_gpu.py -m gpu -q -k "prepared or adam" --timeout 120 --timeout-method thread > $OUT/pytest_form2_$TAG.log 2>&1
rc=$?
tail -2 $OUT/pytest_form2_$TAG.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "form2 pytest ended abnormally ($rc)"; exit $rc; fi
cd /tmp && export TMPDIR=/tmp
for F in 0 1 2; do
  SSQ_K6P_FORM=$F timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $OUT/k6p_${TAG}_$F -o t -- python3 $R/tools/alpha_cold.py 30 > $OUT/k6p_${TAG}_$F.log 2>&1 || { echo "alpha_cold $F failed"; tail -5 $OUT/k6p_${TAG}_$F.log; exit 1; }
  KT=$(find $OUT/k6p_${TAG}_$F -name "*kernel_trace.csv" | head -1)
  python3 $R/tools/trace_avg.py "$KT" alpha_bwd shift_fwd --groups=5 > $OUT/k6p_${TAG}_$F.txt 2>&1
  rm -f "$KT"
  cat $OUT/k6p_${TAG}_$F.txt
done
cd $R
for F in 1 2; do
  SSQ_K6P_FORM=$F timeout -k 10 300 python bench.py --no-cpu-baseline --no-validate --steps 20 --warmup 5 --recon-iters 100 > $OUT/bench_${TAG}_$F.log 2>&1 || { echo "bench $F failed"; tail -5 $OUT/bench_${TAG}_$F.log; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['recon']['resnet18_all_blocks_iters_per_s'], d['recon']['iters_per_s'])" $OUT/bench_${TAG}_$F.log $F
done
exit 0
