R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
TAG=${1:-whole}
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -q -x --timeout 120 --timeout-method thread -k "prepared or adashift" > $OUT/pytest_$TAG.log 2>&1 || { tail -30 $OUT/pytest_$TAG.log; exit 1; }
tail -2 $OUT/pytest_$TAG.log
for co in 0 64 128 256; do
  SSQ_PREP_WHOLE_CO=$co timeout -k 10 120 python tools/adashift_bench.py --blocks > $OUT/ada_${TAG}_$co.log 2>&1 || { tail $OUT/ada_${TAG}_$co.log; exit 1; }
  echo "== WHOLE_CO=$co"; cat $OUT/ada_${TAG}_$co.log | grep -v amdgpu.ids
done
