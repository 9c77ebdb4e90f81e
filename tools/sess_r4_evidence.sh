#!/bin/bash
# Round-end evidence at the tree's kernels: GPU suite + smoke, the bench line, a rocprofv3
# kernel trace of the bench (K1 launch stats, the recon roofline JSON, the iteration
# anatomy), the two PMC passes (HBM traffic JSON), the end-to-end calibration profile.
# Every JSON carries the csrc hash it was measured at (and SSQ_GIT_SHA when passed).
# Usage (via gpurun): SSQ_GIT_SHA=<sha> bash tools/sess_r4_evidence.sh TAG
TAG=${1:-r4e}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
SSQ_PARITY_LOG=$OUT/parity_$TAG.jsonl timeout -k 10 500 python -u -m pytest tests -m gpu -q --maxfail 10 --timeout 120 --timeout-method thread > $OUT/pytest_$TAG.log 2>&1
rc=$?
echo "pytest rc=$rc" >> $OUT/pytest_$TAG.log
tail -2 $OUT/pytest_$TAG.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest ended abnormally ($rc)"; exit $rc; fi
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke_$TAG.log 2>&1 || { echo "smoke failed"; tail -20 $OUT/smoke_$TAG.log; exit 1; }
tail -1 $OUT/smoke_$TAG.log
timeout -k 10 600 python bench.py > $OUT/bench_$TAG.log 2>&1 || { echo "bench failed"; tail -20 $OUT/bench_$TAG.log; exit 1; }
tail -1 $OUT/bench_$TAG.log | cut -c1-300
cd /tmp && export TMPDIR=/tmp
# K6p A/B with cold caches: thread-column everywhere (0), the default per-channel form (3),
# and the per-channel form without its row cap (3, SSQ_K6P_CHAN_CO=4096)
for V in "0 256" "3 256" "3 4096"; do
  set -- $V
  SSQ_K6P_FORM=$1 SSQ_K6P_CHAN_CO=$2 timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $OUT/k6p_${TAG}_$1_$2 -o t -- python3 $R/tools/alpha_cold.py 30 > $OUT/k6p_${TAG}_$1_$2.log 2>&1 || { echo "alpha_cold $V failed"; tail -5 $OUT/k6p_${TAG}_$1_$2.log; exit 1; }
  KT=$(find $OUT/k6p_${TAG}_$1_$2 -name "*kernel_trace.csv" | head -1)
  python3 $R/tools/trace_avg.py "$KT" alpha_bwd --groups=5 > $OUT/k6p_${TAG}_$1_$2.txt 2>&1
  rm -f "$KT"
done
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$TAG -o bench -- python3 $R/bench.py --no-cpu-baseline --no-validate --recon-iters 100 > $OUT/prof_bench_$TAG.log 2>&1 || { echo "rocprof failed"; tail -20 $OUT/prof_bench_$TAG.log; exit 1; }
KT=$(find $OUT/prof_$TAG -name "*kernel_trace.csv" | head -1)
python3 $R/tools/k1_trace_stats.py "$KT" > $OUT/k1_trace_$TAG.json 2>&1
python3 $R/tools/recon_roofline.py "$KT" $OUT/recon_roofline_$TAG.json > $OUT/recon_roofline_$TAG.txt 2>&1
python3 $R/tools/trace_iter.py "$KT" > $OUT/iter_anatomy_$TAG.txt 2>&1
rm -f "$KT"
head -1 $OUT/recon_roofline_$TAG.txt | cut -c1-300
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch_$TAG -o f -- python3 $R/bench.py --no-recon --no-validate --no-cpu-baseline --steps 3 --warmup 1 > $OUT/pmc_fetch_$TAG.log 2>&1 || { echo "fetch pass failed"; tail -20 $OUT/pmc_fetch_$TAG.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write_$TAG -o w -- python3 $R/bench.py --no-recon --no-validate --no-cpu-baseline --steps 3 --warmup 1 > $OUT/pmc_write_$TAG.log 2>&1 || { echo "write pass failed"; tail -20 $OUT/pmc_write_$TAG.log; exit 1; }
python3 $R/tools/pmc_traffic.py $OUT/pmc_fetch_$TAG $OUT/pmc_write_$TAG $OUT/pmc_traffic_$TAG.json > /dev/null 2>&1
find $OUT/pmc_fetch_$TAG $OUT/pmc_write_$TAG -name "*counter_collection.csv" -delete
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print({k: v.get('hbm_bytes_per_launch') for k, v in d.items() if isinstance(v, dict) and 'hbm_bytes_per_launch' in v})" $OUT/pmc_traffic_$TAG.json
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/e2eprof -o e2e -- python3 $R/main_imagenet.py --arch resnet18 --n_bits_w 2 --n_bits_a 4 --weight 1.0 --bias_cal True --bias_ch_quant True > $OUT/e2e_prof_$TAG.log 2>&1 || { echo "e2e failed"; tail -20 $OUT/e2e_prof_$TAG.log; exit 1; }
cp $(find /tmp/e2eprof -name "*kernel_stats.csv" | head -1) $OUT/e2e_kernel_stats_$TAG.csv
grep "calibration finished" $OUT/e2e_prof_$TAG.log | cut -c1-200
# the same calibration unprofiled (its wall time), the act phase's iteration anatomy and
# the short end-to-end runs of the other model families
cd $R
timeout -k 10 600 python main_imagenet.py --arch resnet18 --n_bits_w 2 --n_bits_a 4 --weight 1.0 --bias_cal True --bias_ch_quant True > $OUT/e2e_$TAG.log 2>&1 || { echo "e2e failed"; tail -20 $OUT/e2e_$TAG.log; exit 1; }
grep "calibration finished" $OUT/e2e_$TAG.log | cut -c1-160
SSQ_BRECQ_FAST=0 timeout -k 10 600 python main_imagenet.py --arch resnet18 --n_bits_w 2 --n_bits_a 4 --weight 1.0 --bias_cal True --bias_ch_quant True > $OUT/e2e_brecq_plain_$TAG.log 2>&1 || { echo "e2e (plain BRECQ loop) failed"; tail -20 $OUT/e2e_brecq_plain_$TAG.log; exit 1; }
grep "calibration finished" $OUT/e2e_brecq_plain_$TAG.log | cut -c1-160
bash tools/act_anatomy.sh $TAG || exit 1
cd $R
bash tools/e2e_session.sh $TAG || exit 1
exit 0
