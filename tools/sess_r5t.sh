#!/bin/bash
# r5t A/B: the K13 forward with one channel lookup per float4 (SSQ_K13_PLANE4=1) vs per
# element (0): the act phase's anatomy ABAB (tools/act_anatomy.sh), then the kernel tests.
TAG=${1:-r5t}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -q -k "epilogue or bias_act" --timeout 120 --timeout-method thread > $OUT/pytest_$TAG.log 2>&1 || { echo "tests failed"; tail -20 $OUT/pytest_$TAG.log; exit 1; }
tail -1 $OUT/pytest_$TAG.log
for rep in 1 2; do
for P in 1 0; do
  SSQ_K13_PLANE4=$P bash tools/act_anatomy.sh ${TAG}_p${P}_$rep > /dev/null || exit 1
  echo "== PLANE4=$P rep $rep"; grep -A6 "^---" $OUT/act_anatomy_${TAG}_p${P}_$rep.txt | grep "^---\|bias_act" | cut -c1-80
  rm -f $OUT/act_trace_${TAG}_p${P}_$rep.csv.gz
done
done
exit 0
