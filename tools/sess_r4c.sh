#!/bin/bash
# r4 session: GPU suite (default K6p form 3), the form-1 prepared tests, K6p forms 0-3 A/B,
# recon per form, world-2 gloo rehearsal.
TAG=${1:-r4c}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
SSQ_PARITY_LOG=$OUT/parity_$TAG.jsonl timeout -k 10 500 python -u -m pytest tests -m gpu -q --maxfail 10 --timeout 120 --timeout-method thread > $OUT/pytest_$TAG.log 2>&1
rc=$?
echo "pytest rc=$rc" >> $OUT/pytest_$TAG.log
tail -3 $OUT/pytest_$TAG.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest ended abnormally ($rc)"; exit $rc; fi
SSQ_K6P_FORM=1 timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_recon_gpu.py -m gpu -q -k "prepared or adam or fused" --timeout 120 --timeout-method thread > $OUT/pytest_form2_$TAG.log 2>&1
rc=$?
tail -2 $OUT/pytest_form2_$TAG.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "form2 pytest ended abnormally ($rc)"; exit $rc; fi
cd /tmp && export TMPDIR=/tmp
for F in 0 1 2 3; do
  SSQ_K6P_FORM=$F timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $OUT/k6p_${TAG}_$F -o t -- python3 $R/tools/alpha_cold.py 30 > $OUT/k6p_${TAG}_$F.log 2>&1 || { echo "alpha_cold $F failed"; tail -5 $OUT/k6p_${TAG}_$F.log; exit 1; }
  KT=$(find $OUT/k6p_${TAG}_$F -name "*kernel_trace.csv" | head -1)
  python3 $R/tools/trace_avg.py "$KT" alpha_bwd --groups=5 > $OUT/k6p_${TAG}_$F.txt 2>&1
  rm -f "$KT"
  cat $OUT/k6p_${TAG}_$F.txt
done
cd $R
for F in 1 3; do
  SSQ_K6P_FORM=$F timeout -k 10 300 python bench.py --no-cpu-baseline --no-validate --steps 20 --warmup 5 --recon-iters 100 > $OUT/bench_${TAG}_$F.log 2>&1 || { echo "bench $F failed"; tail -5 $OUT/bench_${TAG}_$F.log; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['recon']['resnet18_all_blocks_iters_per_s'], d['recon']['iters_per_s'])" $OUT/bench_${TAG}_$F.log $F
done
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 20 --warmup 5 --dist-backend gloo --no-cpu-baseline --no-validate --recon-iters 60 > $OUT/dist2_$TAG.log 2>&1 || { echo "dist2 failed"; tail -20 $OUT/dist2_$TAG.log; exit 1; }
tail -1 $OUT/dist2_$TAG.log | cut -c1-400
exit 0
