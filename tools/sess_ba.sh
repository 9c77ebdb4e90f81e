# r3: K13 forward (bias_act) and the RPW=1 epilogue backward with loads issued ahead -- its parity tests, its duration in the
# recon loop under rocprofv3, then bench.py at the driver's step counts (20 / 5) and default.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
TAG=${1:-ba}
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_recon_gpu.py -m gpu -q -x --timeout 120 --timeout-method thread -k "bias_act or epilogue or fused or recon" > $OUT/pytest_$TAG.log 2>&1 || { grep -E "^E |FAILED" $OUT/pytest_$TAG.log | head -30; exit 1; }
tail -1 $OUT/pytest_$TAG.log
for i in 1 2 3; do
  timeout -k 10 150 python bench.py --steps 20 --warmup 5 --no-recon --no-validate --no-cpu-baseline > $OUT/b20_${TAG}_$i.json 2>$OUT/b20_${TAG}_$i.err || { tail $OUT/b20_${TAG}_$i.err; exit 1; }
done
timeout -k 10 150 python bench.py --no-recon --no-validate --no-cpu-baseline > $OUT/b100_$TAG.json 2>$OUT/b100_$TAG.err || { tail $OUT/b100_$TAG.err; exit 1; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/ba_$TAG$RANDOM -o ba -- python3 $R/tools/recon_blocks.py 100 ${BLOCKS:-layer1.0 layer2.1 layer3.1} > $OUT/ba_$TAG.log 2>&1 || { tail $OUT/ba_$TAG.log; exit 1; }
KT=$(find $OUT -path "*ba_$TAG*" -name "*kernel_trace.csv" | head -1)
tail -1 $OUT/ba_$TAG.log
python3 $R/tools/trace_avg.py "$KT" bias_act_kernel epilogue_bwd_rows gather --groups=${NG:-3} > $OUT/ba_avg_$TAG.txt; rm -f "$KT"
cat $OUT/ba_avg_$TAG.txt
