R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
bash tools/session.sh r6f tests || exit 1
timeout -k 10 400 python tools/wgrad_grouped_probe.py > $OUT/wgrad_grouped.log 2>&1 || { echo "probe failed"; tail -3 $OUT/wgrad_grouped.log; exit 1; }
grep -v amdgpu.ids $OUT/wgrad_grouped.log | cut -c1-400
bash tools/session.sh r6f cfgtrace
