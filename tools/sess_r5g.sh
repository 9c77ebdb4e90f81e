#!/bin/bash
# r5g: the new / changed tests (K19 backward, in-place rows), the fc loop rates + anatomy
# (sess_r5d.sh), then the end-to-end ResNet-18 flow and the act phase's anatomy (sess_e2e.sh).
TAG=${1:-r5g}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
bash tools/sess_r5d.sh $TAG "fc_fused or fc_recon or specials or rows or knobs or identity_block or epilogue" || exit $?
bash tools/sess_e2e.sh $TAG || exit $?
