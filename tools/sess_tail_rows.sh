#!/bin/bash
# Fused tail (ssq_epilogue_loss_bwd) on 7x7 scalar rows: one row per wave (SSQ_EPI_MULTI_ROW=1)
# vs four (=3, the downsample-folding RES 2 form included).  The fused-tail and loop tests
# under =3, then ResNet-18 layer4.0 / layer4.1's fused loop under rocprofv3 in each mode.
# (r4: the knob value 3 was removed again after this A/B, profiles/r4_tail_rows_ab.txt)
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
TAG=${1:-tr}
SSQ_EPI_MULTI_ROW=3 timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_recon_gpu.py tests/test_realshape_gpu.py -m gpu -q -x --timeout 120 --timeout-method thread > $OUT/pytest_$TAG.log 2>&1 || { grep -E "^E |FAILED" $OUT/pytest_$TAG.log | head -30; tail -3 $OUT/pytest_$TAG.log; exit 1; }
tail -1 $OUT/pytest_$TAG.log
cd /tmp && export TMPDIR=/tmp
for m in 1 3 1 3; do
  D=$OUT/tail_$TAG${m}_$RANDOM
  SSQ_EPI_MULTI_ROW=$m timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $D -o t -- python3 $R/tools/recon_blocks.py 100 layer4.0 layer4.1 > $D.log 2>&1 || { echo "run $m failed"; tail $D.log; exit 1; }
  KT=$(find $D -name "*kernel_trace.csv" | head -1)
  echo "multi_row=$m $(tail -1 $D.log)"
  python3 $R/tools/trace_avg.py "$KT" epilogue_bwd_rows --groups=2
  rm -f "$KT"
done
