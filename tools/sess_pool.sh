# r3: the stem's max-pool on ssq_maxpool2d_fwd (SSQ_MAXPOOL) on and off in one session: its
# parity test and the validation tests, then bench.py's validation line alternating.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
TAG=${1:-pool}
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_recon2_gpu.py tests/test_dp_gpu.py -m gpu -q -x --timeout 120 --timeout-method thread -k "maxpool or valid" > $OUT/pytest_$TAG.log 2>&1 || { grep -E "^E |FAILED" $OUT/pytest_$TAG.log | head -30; exit 1; }
tail -1 $OUT/pytest_$TAG.log
for v in 1 0 1 0; do
  SSQ_POOL_PAIR=$v timeout -k 10 300 python bench.py --no-cpu-baseline --no-recon --steps 20 --warmup 5 > $OUT/bpool_${TAG}_$v.log 2>&1 || { tail $OUT/bpool_${TAG}_$v.log; exit 1; }
  python3 - "$OUT/bpool_${TAG}_$v.log" $v <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(json.dumps({"pool_pair": sys.argv[2], "val_img_s": d["validation"]["images_per_s"],
                  "val_ms": d["validation"]["ms_per_batch"]}))
PY
done
