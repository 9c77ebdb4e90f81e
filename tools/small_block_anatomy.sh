#!/bin/bash
# Wall vs GPU-busy time per fused-loop iteration on small blocks (MobileNetV2, RegNetX):
# rocprofv3 kernel traces of tools/block_anatomy.py + tools/trace_iter.py.
TAG=${1:-run}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for AB in "mobilenetv2 features.2" "mobilenetv2 features.14" "regnetx_3200m s3.b2" "resnet50 layer4.1"; do
  set -- $AB
  N=$(echo "$1_$2" | tr '.' '_')
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/prof_sb_${TAG}_$N -o t -- python3 $R/tools/block_anatomy.py $1 $2 200 1 > $OUT/sb_${TAG}_$N.log 2>&1 || { echo "$AB failed"; tail -5 $OUT/sb_${TAG}_$N.log; exit 1; }
  KT=$(find $OUT/prof_sb_${TAG}_$N -name "*kernel_trace.csv" | head -1)
  python3 $R/tools/trace_iter.py "$KT" > $OUT/sb_anatomy_${TAG}_$N.txt 2>&1
  rm -f "$KT"
  echo "$AB: $(tail -1 $OUT/sb_${TAG}_$N.log | cut -c1-150)"
  grep -- "^---" $OUT/sb_anatomy_${TAG}_$N.txt | head -3
done
