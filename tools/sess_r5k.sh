#!/bin/bash
# r5k: the full GPU suite + smoke, then the 16-lanes-per-row epilogue form (SSQ_EPI_G16) A/B
# in bench.py's recon loops (ABAB, per-block iterations/s), then the recon roofline trace.
TAG=${1:-r5k}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
bash tools/sess_tests.sh $TAG
rc=$?
[ $rc -gt 1 ] && exit $rc
for V in 1 0 1 0; do
  SSQ_EPI_G16=$V timeout -k 10 300 python bench.py --no-cpu-baseline --no-validate --steps 3 --warmup 1 > $OUT/g16_${TAG}_$V.log 2>&1 || { echo "bench $V failed"; tail -5 $OUT/g16_${TAG}_$V.log; exit 1; }
  tail -1 $OUT/g16_${TAG}_$V.log | python -c "import json,sys; d=json.loads(sys.stdin.read())['recon']; print('SSQ_EPI_G16=$V', json.dumps(d['iters_per_s']), d['resnet18_all_blocks_iters_per_s'])"
done
cd /tmp && export TMPDIR=/tmp
for V in 1 0; do
  SSQ_EPI_G16=$V timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d $OUT/prof_g16_${TAG}_$V -o bench -- python3 $R/bench.py --no-cpu-baseline --no-validate --recon-iters 100 > $OUT/prof_g16_${TAG}_$V.log 2>&1 || { echo "rocprof $V failed"; tail -20 $OUT/prof_g16_${TAG}_$V.log; exit 1; }
  KT=$(find $OUT/prof_g16_${TAG}_$V -name "*kernel_trace.csv" | head -1)
  python3 $R/tools/recon_roofline.py "$KT" $OUT/recon_roofline_${TAG}_$V.json > $OUT/recon_roofline_${TAG}_$V.txt 2>&1
  rm -f "$KT"
  echo "G16=$V $(head -1 $OUT/recon_roofline_${TAG}_$V.txt | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["us_per_iteration"], d["frac"])')"
done
exit $rc
