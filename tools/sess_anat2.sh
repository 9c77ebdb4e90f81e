R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
TAG=${1:-a2}
BLK=${2:-layer2.0}
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $OUT/anat_$TAG -o t -- python3 $R/tools/block_anatomy.py resnet18 $BLK 60 1 256 > $OUT/anat_$TAG.log 2>&1 || { tail $OUT/anat_$TAG.log; exit 1; }
KT=$(find $OUT/anat_$TAG -name "*kernel_trace.csv" | head -1)
python3 $R/tools/trace_iter.py "$KT" full > $OUT/anat_${TAG}_full.txt 2>&1
rm -f "$KT"
head -32 $OUT/anat_${TAG}_full.txt | cut -c1-170
