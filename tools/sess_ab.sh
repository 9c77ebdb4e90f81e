# A/B of an environment knob on the deterministic-solver fused recon loop (tools/recon_blocks.py):
#   KNOB=NAME VALUES="a b a b" BLOCKS="layer4.0 layer4.1" bash tools/sess_ab.sh TAG
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
TAG=${1:-ab}
for v in $VALUES; do
  env $KNOB=$v timeout -k 10 300 python -u tools/recon_blocks.py ${ITERS:-200} $BLOCKS > $OUT/ab_$TAG.$v.log 2>&1 || { echo "$KNOB=$v failed"; tail $OUT/ab_$TAG.$v.log; exit 1; }
  echo "$KNOB=$v $(tail -1 $OUT/ab_$TAG.$v.log)"
done
