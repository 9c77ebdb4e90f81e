#!/bin/bash
# PMC pass over K17's band kernel (ssq_conv_wgrad, auto form) on ResNet-18 shapes.
# Usage (via gpurun): bash tools/pmc_band.sh TAG
TAG=${1:-run}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"
for shape in "64 56 64 3 1 1 1" "256 14 256 3 1 1 1" "512 7 512 3 1 1 1"; do
  tag=$(echo $shape | tr ' ' '_')
  timeout -s KILL 90 rocprofv3 --pmc $P1 --output-format csv -d $OUT/pmc_band_${TAG}_$tag -o p -- python3 $R/tools/wgrad_one.py $shape 5 > $OUT/pmc_band_${TAG}_$tag.log 2>&1 || { echo "pmc failed $shape"; tail -5 $OUT/pmc_band_${TAG}_$tag.log; exit 1; }
done
echo ok
