# r3: only the gradient / real-shape parity tests (verbose), with their parity log.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
TAG=${1:-nt}
rm -f $OUT/parity_$TAG.jsonl
SSQ_PARITY_LOG=$OUT/parity_$TAG.jsonl timeout -k 10 600 python -u -m pytest tests/test_grads_gpu.py tests/test_realshape_gpu.py -m gpu -v --timeout 300 --timeout-method thread > $OUT/pytest_new_$TAG.log 2>&1
rc=$?
tail -20 $OUT/pytest_new_$TAG.log
exit $rc
