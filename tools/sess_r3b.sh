# r3: the new gradient / real-shape parity tests first (verbose), then the whole GPU suite.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
TAG=${1:-r3b}
rm -f $OUT/parity_$TAG.jsonl
SSQ_PARITY_LOG=$OUT/parity_$TAG.jsonl timeout -k 10 600 python -u -m pytest tests/test_grads_gpu.py tests/test_realshape_gpu.py -m gpu -v --timeout 300 --timeout-method thread > $OUT/pytest_new_$TAG.log 2>&1
rc=$?
tail -30 $OUT/pytest_new_$TAG.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest ended abnormally ($rc)"; exit $rc; fi
SSQ_PARITY_LOG=$OUT/parity_all_$TAG.jsonl timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu_$TAG.log 2>&1
rc2=$?
tail -5 $OUT/pytest_gpu_$TAG.log
exit $rc2
