# r3: multi-row epilogue backward -- epilogue / fused-tail / loop parity tests, then the
# small-plane blocks' loop under rocprofv3 with the knob on and off.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
TAG=${1:-epi}
[ -z "$SKIP_TESTS" ] && timeout -k 10 500 python -u -m pytest tests/test_kernels_gpu.py tests/test_recon_gpu.py tests/test_recon2_gpu.py tests/test_realshape_gpu.py -m gpu -q -x --timeout 120 --timeout-method thread > $OUT/pytest_$TAG.log 2>&1
rc=$?; [ -z "$SKIP_TESTS" ] && tail -2 $OUT/pytest_$TAG.log; [ -n "$SKIP_TESTS" ] && rc=0
if [ $rc -ne 0 ]; then grep -E "^E |FAILED" $OUT/pytest_$TAG.log | head -30; exit 1; fi
cd /tmp && export TMPDIR=/tmp
for m in ${MODES:-1 0}; do
  SSQ_EPI_MULTI_ROW=$m timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/epi_$TAG$m$RANDOM -o epi -- python3 $R/tools/recon_blocks.py 100 ${BLOCKS:-layer1.0 layer2.1 layer3.1 layer4.1} > $OUT/epi_$TAG$m.log 2>&1 || { echo "run $m failed"; tail $OUT/epi_$TAG$m.log; exit 1; }
  KT=$(find $OUT -path "*epi_$TAG$m*" -name "*kernel_trace.csv" | head -1)
  echo "multi_row=$m $(tail -1 $OUT/epi_$TAG$m.log)"
  python3 $R/tools/trace_avg.py "$KT" epilogue_bwd_rows --groups=${NG:-4} > $OUT/epi_avg_$TAG$m.txt; rm -f "$KT"
  cat $OUT/epi_avg_$TAG$m.txt
done
