# r3: where the K17 band kernel's cycles go on ResNet-18 layer1's 3x3 conv (64x56x56,
# batch 32): wave-cycle buckets, MFMA busy cycles and the effective clock, one rocprofv3
# --pmc pass each (SQ <= 8, GRBM <= 2 counters per pass), then the kernel trace.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
TAG=${1:-band}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
SHAPE=${SHAPE:-64 56 64 3 1 1 1}
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $OUT/pmc_$TAG -o p1 -- python3 $R/tools/wgrad_one.py $SHAPE 20 > $OUT/pmc_$TAG.log 2>&1 || { echo "pmc pass failed"; tail $OUT/pmc_$TAG.log; exit 1; }
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt_$TAG -o kt -- python3 $R/tools/wgrad_one.py $SHAPE 20 >> $OUT/pmc_$TAG.log 2>&1 || { echo "trace failed"; exit 1; }
python3 $R/tools/pmc_summary.py $OUT/pmc_$TAG $OUT/kt_$TAG wgrad_band_stage1 | tee $OUT/pmc_summary_$TAG.txt
