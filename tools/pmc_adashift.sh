#!/bin/bash
# PMC passes (FETCH_SIZE, WRITE_SIZE; separate runs) over the recon iteration's ssq kernels
# at the ResNet-18 block shapes (tools/adashift_bench.py --blocks: multi-segment adaShift
# forward / backward), plus SQ busy counters.  Usage (via gpurun): bash tools/pmc_adashift.sh TAG
TAG=${1:-run}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for pass in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE"; do
  tag=$(echo $pass | cut -d' ' -f1)
  timeout -s KILL 120 rocprofv3 --pmc $pass --output-format csv -d $OUT/pmc_ada_${TAG}_$tag -o p -- python3 $R/tools/adashift_bench.py --blocks > $OUT/pmc_ada_${TAG}_$tag.log 2>&1 || { echo "pmc pass $tag failed"; tail -5 $OUT/pmc_ada_${TAG}_$tag.log; exit 1; }
done
python3 $R/tools/pmc_ssq_summary.py $OUT/pmc_ada_${TAG}_FETCH_SIZE $OUT/pmc_ada_${TAG}_WRITE_SIZE $OUT/pmc_ada_${TAG}_SQ_WAVE_CYCLES > $OUT/pmc_ada_${TAG}.json
cat $OUT/pmc_ada_${TAG}.json
