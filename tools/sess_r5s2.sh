#!/bin/bash
# The torch-native kernel in the downsample blocks' recon iteration: one block's loop under
# the kernel tracer, full kernel names per iteration (tools/trace_iter.py full).
TAG=${1:-r5s2}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/prof_$TAG -o t -- python3 -c "
import sys, torch; sys.path.insert(0, '$R')
torch.backends.cudnn.benchmark, torch.backends.cudnn.deterministic = False, True
from shiftedscalequantization_amd.recon_bench import run_block
print(run_block(torch.device('cuda'), 'layer2.0', iters=60)['ips'])
" > $OUT/prof_$TAG.log 2>&1 || { echo "trace failed"; tail -20 $OUT/prof_$TAG.log; exit 1; }
KT=$(find $OUT/prof_$TAG -name "*kernel_trace.csv" | head -1)
python3 $R/tools/trace_iter.py "$KT" full > $OUT/anat_$TAG.txt 2>&1
rm -f "$KT"
tail -1 $OUT/prof_$TAG.log
grep -A20 "^---" $OUT/anat_$TAG.txt | tail -21 | cut -c1-230
exit 0
