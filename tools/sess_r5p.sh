#!/bin/bash
# r5p: the epilogue / act-quant / BRECQ tests after the exact reciprocal division in the K13
# act-quant math, then the act phase's anatomy (compare profiles/r5_act_anatomy_r5ev2.txt).
TAG=${1:-r5p}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
bash tools/sess_tests.sh $TAG "epilogue or bias_act or brecq or rows or knobs or identity_block or fused_tail or quant_block or fq" || exit $?
bash tools/act_anatomy.sh $TAG || exit 1
grep -A4 -- "---" gpurun_out/act_anatomy_$TAG.txt | head -30 | cut -c1-110
