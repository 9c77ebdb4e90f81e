# r3: the band kernel at 8 waves (two per SIMD, taps split) against 4: the fp64 wgrad
# parity tests and the recon loop tests with SSQ_BAND_WAVES=8, then tools/band_ab.py
# alternating the two forms in one session.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
TAG=${1:-bw8}
SSQ_BAND_WAVES=8 timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_recon_gpu.py -m gpu -q -x --timeout 120 --timeout-method thread -k "wgrad or recon" > $OUT/pytest_$TAG.log 2>&1 || { grep -E "^E |FAILED" $OUT/pytest_$TAG.log | head -30; exit 1; }
tail -1 $OUT/pytest_$TAG.log
for v in 4 8 4 8; do
  SSQ_BAND_WAVES=$v timeout -k 10 120 python tools/band_ab.py w$v >> $OUT/band_ab_$TAG.jsonl 2>&1 || { echo "band_ab $v failed"; tail $OUT/band_ab_$TAG.jsonl; exit 1; }
done
grep -v amdgpu.ids $OUT/band_ab_$TAG.jsonl
