#!/bin/bash
# fc AdaRound loop: unprofiled rate vs the chunk graph's back-to-back replay time (GPU work +
# launch boundaries only), K19 and the unfused launches.
TAG=${1:-fcp}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
for F in 1 0; do
  SSQ_FUSE_FC=$F SSQ_BRECQ_CHUNK=25 timeout -k 10 300 python tools/fc_recon_rate.py > $OUT/fc_probe_${TAG}_f$F.log 2>&1 || { echo "probe $F failed"; tail -5 $OUT/fc_probe_${TAG}_f$F.log; exit 1; }
  echo "fuse=$F $(grep -E 'fc_adaround|chunk_replay' $OUT/fc_probe_${TAG}_f$F.log | tr '\n' ' ')"
done
