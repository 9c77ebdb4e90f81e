#!/bin/bash
# GPU suite + smoke at the tree's kernels (one box session).  Usage: bash tools/sess_tests.sh TAG [pytest -k expr]
TAG=${1:-run}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
K=()
[ -n "$2" ] && K=(-k "$2")
SSQ_PARITY_LOG=$OUT/parity_$TAG.jsonl timeout -k 10 900 python -u -m pytest tests -m gpu -q --maxfail 10 --timeout 120 --timeout-method thread -rs "${K[@]}" > $OUT/pytest_$TAG.log 2>&1
rc=$?
echo "pytest rc=$rc" >> $OUT/pytest_$TAG.log
tail -4 $OUT/pytest_$TAG.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest ended abnormally ($rc)"; exit $rc; fi
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke_$TAG.log 2>&1 || { echo "smoke failed"; tail -20 $OUT/smoke_$TAG.log; exit 1; }
tail -1 $OUT/smoke_$TAG.log
exit $rc
