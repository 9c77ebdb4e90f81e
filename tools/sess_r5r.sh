#!/bin/bash
# r5r: the epilogue-into-im2col test with the reworked kernel (LDS channel operands, 16-B
# stores), then the fold's A/B in bench.py's recon loops (ABAB, per-block iterations/s).
TAG=${1:-r5r}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
bash tools/sess_tests.sh $TAG "into_gemm or fused_epilogue or quant_block" || exit $?
bash tools/sess_epi_gemm_ab.sh $TAG || exit $?
