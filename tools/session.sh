#!/bin/bash
# One GPU box session, parameterised by its steps (replaces the per-round sess_*.sh one-offs).
#
#   bash tools/session.sh TAG STEP [STEP ...]          (via gpurun; outputs in gpurun_out/)
#
# Steps, run in the order given; the first failure, abort, segfault or time limit ends the
# session (no later GPU step runs after it):
#   tests     pytest -m gpu (parity log parity_TAG.jsonl) + smoke()   [TESTS_K: a -k filter]
#   bench     python bench.py (the driver's default line)              -> bench_TAG.log
#   trace     rocprofv3 kernel trace of bench.py: K1 launch stats, the ResNet-18 recon
#             roofline JSON, the iteration anatomy                      -> k1_trace / recon_roofline / iter_anatomy
#   cfgtrace  rocprofv3 kernel trace of BASELINE configs 3-5's loops (tools/recon_configs_trace.py)
#             and their ssq-set rooflines                               -> recon_configs_roofline_TAG.json
#   pmc       the two PMC passes (FETCH_SIZE, WRITE_SIZE) of the q/dq step -> pmc_traffic_TAG.json
#   e2e       main_imagenet.py end to end (ResNet-18 W2A4 --bias_cal --bias_ch_quant), the
#             short runs of ResNet-50 / RegNetX-3200M / MobileNetV2   -> e2e_*_TAG.log
#   act       the BRECQ act phase's iteration anatomy (tools/act_anatomy.sh)
#   fc        the fc AdaRound loop's rate and anatomy (K19)
#   dist2     bench.py --gpus 2 self-launched over gloo (two ranks on the box's GPU)
TAG=${1:?tag}
shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp

fail() { echo "$1"; [ -n "$2" ] && tail -20 "$2"; exit 1; }

step_tests() {
  cd $R
  local K=()
  [ -n "$TESTS_K" ] && K=(-k "$TESTS_K")
  SSQ_PARITY_LOG=$OUT/parity_$TAG.jsonl timeout -k 10 700 python -u -m pytest tests -m gpu -q \
    --maxfail 10 --timeout 200 --timeout-method thread -rs "${K[@]}" > $OUT/pytest_$TAG.log 2>&1
  local rc=$?
  echo "pytest rc=$rc" >> $OUT/pytest_$TAG.log
  tail -3 $OUT/pytest_$TAG.log
  if [ $rc -ne 0 ]; then echo "pytest failed ($rc)"; exit $rc; fi
  timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke_$TAG.log 2>&1 \
    || fail "smoke failed" $OUT/smoke_$TAG.log
  tail -1 $OUT/smoke_$TAG.log
}

step_bench() {
  cd $R
  timeout -k 10 600 python bench.py > $OUT/bench_$TAG.log 2>&1 || fail "bench failed" $OUT/bench_$TAG.log
  tail -1 $OUT/bench_$TAG.log | cut -c1-300
}

step_trace() {
  cd /tmp
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$TAG -o bench \
    -- python3 $R/bench.py --no-cpu-baseline --no-validate --no-recon-configs --recon-iters 100 \
    > $OUT/prof_bench_$TAG.log 2>&1 || fail "rocprof bench failed" $OUT/prof_bench_$TAG.log
  local KT=$(find $OUT/prof_$TAG -name "*kernel_trace.csv" | head -1)
  python3 $R/tools/k1_trace_stats.py "$KT" > $OUT/k1_trace_$TAG.json 2>&1
  python3 $R/tools/recon_roofline.py "$KT" $OUT/recon_roofline_$TAG.json > $OUT/recon_roofline_$TAG.txt 2>&1
  python3 $R/tools/trace_iter.py "$KT" > $OUT/iter_anatomy_$TAG.txt 2>&1
  rm -f "$KT"       # tens of MB: keep the summaries
  head -1 $OUT/recon_roofline_$TAG.txt | cut -c1-300
}

step_cfgtrace() {
  cd /tmp
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/cfgprof_$TAG -o cfg \
    -- python3 $R/tools/recon_configs_trace.py 100 $OUT/cfg_side_$TAG.json \
    > $OUT/cfgprof_$TAG.log 2>&1 || fail "rocprof configs failed" $OUT/cfgprof_$TAG.log
  local KT=$(find $OUT/cfgprof_$TAG -name "*kernel_trace.csv" | head -1)
  python3 $R/tools/recon_roofline.py --configs "$KT" $OUT/cfg_side_$TAG.json \
    $OUT/recon_configs_roofline_$TAG.json > $OUT/recon_configs_roofline_$TAG.txt 2>&1 \
    || fail "configs roofline failed" $OUT/recon_configs_roofline_$TAG.txt
  gzip -c "$KT" > $OUT/cfg_trace_$TAG.csv.gz
  rm -f "$KT"
  cat $OUT/recon_configs_roofline_$TAG.txt | cut -c1-200
}

step_pmc() {
  cd /tmp
  local B="$R/bench.py --no-recon --no-validate --no-cpu-baseline --steps 3 --warmup 1"
  timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch_$TAG -o f \
    -- python3 $B > $OUT/pmc_fetch_$TAG.log 2>&1 || fail "fetch pass failed" $OUT/pmc_fetch_$TAG.log
  timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write_$TAG -o w \
    -- python3 $B > $OUT/pmc_write_$TAG.log 2>&1 || fail "write pass failed" $OUT/pmc_write_$TAG.log
  python3 $R/tools/pmc_traffic.py $OUT/pmc_fetch_$TAG $OUT/pmc_write_$TAG $OUT/pmc_traffic_$TAG.json > /dev/null 2>&1
  find $OUT/pmc_fetch_$TAG $OUT/pmc_write_$TAG -name "*counter_collection.csv" -delete
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print({k: v.get('hbm_bytes_per_launch') for k, v in d.items() if isinstance(v, dict) and 'hbm_bytes_per_launch' in v})" $OUT/pmc_traffic_$TAG.json
}

step_e2e() {
  cd $R
  local A="--arch resnet18 --n_bits_w 2 --n_bits_a 4 --weight 1.0 --bias_cal True --bias_ch_quant True"
  timeout -k 10 600 python main_imagenet.py $A > $OUT/e2e_$TAG.log 2>&1 || fail "e2e failed" $OUT/e2e_$TAG.log
  grep "calibration finished" $OUT/e2e_$TAG.log | cut -c1-160
  bash tools/e2e_session.sh $TAG || exit 1
}

step_act() {
  cd $R
  bash tools/act_anatomy.sh $TAG || exit 1
}

step_fc() {
  cd $R
  timeout -k 10 300 python tools/fc_recon_rate.py > $OUT/fc_rate_$TAG.log 2>&1 || fail "fc rate failed" $OUT/fc_rate_$TAG.log
  grep fc_adaround $OUT/fc_rate_$TAG.log
  cd /tmp
  timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $OUT/prof_fc_$TAG -o fc \
    -- python3 $R/tools/fc_recon_rate.py > $OUT/prof_fc_$TAG.log 2>&1 || fail "rocprof fc failed" $OUT/prof_fc_$TAG.log
  local KT=$(find $OUT/prof_fc_$TAG -name "*kernel_trace.csv" | head -1)
  MARKER=fc_fwd_loss python3 $R/tools/trace_iter.py "$KT" > $OUT/fc_anatomy_$TAG.txt 2>&1
  rm -f "$KT"
}

step_dist2() {
  cd $R
  timeout -k 10 400 python bench.py --gpus 2 --dist-backend gloo --steps 20 --warmup 5 --no-cpu-baseline \
    --no-recon-configs --recon-iters 30 > $OUT/dist2_$TAG.log 2>&1 || fail "dist2 failed" $OUT/dist2_$TAG.log
  tail -1 $OUT/dist2_$TAG.log | cut -c1-200
}

for s in "$@"; do
  echo "== $s"
  type step_$s > /dev/null 2>&1 || { echo "unknown step $s"; exit 2; }
  step_$s
done
exit 0
