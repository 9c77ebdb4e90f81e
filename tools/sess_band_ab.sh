# r3: K17 band-kernel A/B in one session: the fp64 wgrad parity tests and the recon loop
# tests on the new build, then tools/band_ab.py alternating the base build (ab/) and the
# new one (in-tree).  Make the base first, e.g.: git stash; python -c "import __graft_entry__
# as g; g.build()"; mkdir -p ab; cp shiftedscalequantization_amd/libssq.so ab/libssq_base.so;
# git stash pop; rebuild.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
TAG=${1:-bab}
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_recon_gpu.py -m gpu -q -x --timeout 120 --timeout-method thread -k "wgrad or recon" > $OUT/pytest_$TAG.log 2>&1 || { grep -E "^E |FAILED" $OUT/pytest_$TAG.log | head -30; exit 1; }
tail -1 $OUT/pytest_$TAG.log
for v in base new base new; do
  if [ $v = base ]; then L=$R/ab/libssq_base.so; else L=$R/shiftedscalequantization_amd/libssq.so; fi
  SSQ_LIB=$L timeout -k 10 120 python tools/band_ab.py $v >> $OUT/band_ab_$TAG.jsonl 2>&1 || { echo "band_ab $v failed"; tail $OUT/band_ab_$TAG.jsonl; exit 1; }
done
cat $OUT/band_ab_$TAG.jsonl
