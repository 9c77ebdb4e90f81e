#!/bin/bash
# PMC passes (FETCH_SIZE, WRITE_SIZE, SQ busy; separate runs) over the recon loop itself:
# block_recon_fused_shiftedScale on ResNet-18 BLOCK (default layer1.0), reference-faithful
# solvers, 30 iterations, 256-sample cache -- every ssq kernel of the iteration (gather,
# prepared adaShift, epilogues, lp_loss, K17 wgrad, Adam) at its real shapes.
# Usage (via gpurun): bash tools/pmc_recon.sh TAG [BLOCK]
TAG=${1:-run}
BLOCK=${2:-layer1.0}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for pass in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE"; do
  tag=$(echo $pass | cut -d' ' -f1)
  timeout -s KILL 150 rocprofv3 --pmc $pass --output-format csv -d $OUT/pmc_rec_${TAG}_$tag -o p -- python3 $R/tools/block_anatomy.py resnet18 $BLOCK 30 1 256 > $OUT/pmc_rec_${TAG}_$tag.log 2>&1 || { echo "pmc pass $tag failed"; tail -5 $OUT/pmc_rec_${TAG}_$tag.log; exit 1; }
done
python3 $R/tools/pmc_ssq_summary.py $OUT/pmc_rec_${TAG}_FETCH_SIZE $OUT/pmc_rec_${TAG}_WRITE_SIZE $OUT/pmc_rec_${TAG}_SQ_WAVE_CYCLES > $OUT/pmc_rec_${TAG}.json
# the raw per-dispatch CSVs are large; keep the summary
find $OUT -path "*pmc_rec_${TAG}_*" -name "*counter_collection.csv" -delete
echo "pmc summary: $OUT/pmc_rec_${TAG}.json"
