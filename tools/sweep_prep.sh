cd $GRAFT_REPO_ROOT
for w in 1536 768 3072; do for r in 8 16 4; do
SSQ_PREP_WGS=$w SSQ_PREP_ROWS=$r timeout -k 10 60 python -u tools/adashift_bench.py --blocks >> gpurun_out/sweep_prep.log 2>&1 || exit 1
done; done
