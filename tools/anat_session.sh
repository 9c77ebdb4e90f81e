
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/anat
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for spec in "mobilenetv2 features.2" "mobilenetv2 features.4" "regnetx_3200m s2.b1" "resnet50 layer1.0"; do
  set -- $spec
  tag=$1_$2
  timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $OUT/$tag -o t -- python3 $R/tools/block_anatomy.py $1 $2 60 1 256 > $OUT/$tag.log 2>&1
  tail -1 $OUT/$tag.log
  KT=$(find $OUT/$tag -name "*kernel_trace.csv" | head -1)
  python3 $R/tools/trace_iter.py "$KT" > $OUT/$tag.anat.txt 2>&1 || true
  rm -f "$KT"
done
