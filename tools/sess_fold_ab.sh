#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_recon_gpu.py tests/test_recon2_gpu.py tests/test_grads_gpu.py tests/test_dp_gpu.py -m gpu -q --maxfail 10 --timeout 120 --timeout-method thread > $OUT/pytest_fold.log 2>&1
rc=$?
tail -3 $OUT/pytest_fold.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest abnormal $rc"; exit $rc; fi
cd /tmp && export TMPDIR=/tmp
for F in 1 0; do
  SSQ_FOLD_RESIDUAL=$F timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/prof_fold_$F -o t -- python3 $R/tools/block_anatomy.py resnet18 layer2.0 200 1 > $OUT/fold_$F.log 2>&1 || { echo "anatomy $F failed"; tail -5 $OUT/fold_$F.log; exit 1; }
  KT=$(find $OUT/prof_fold_$F -name "*kernel_trace.csv" | head -1)
  python3 $R/tools/trace_iter.py "$KT" > $OUT/fold_anatomy_$F.txt 2>&1
  rm -f "$KT"
  echo "FOLD=$F"; head -16 $OUT/fold_anatomy_$F.txt | cut -c1-120
done
