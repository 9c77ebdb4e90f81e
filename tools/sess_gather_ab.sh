#!/bin/bash
# BRECQ act phase: the batch input and the cached block-input convs' rows gathered two per
# launch (block_recon.GATHER_ONCE) vs one launch each.  The loop tests, then the default
# end-to-end flow with it on and off (block losses must print identically), then the act
# phase's iteration anatomy with it on.
set -o pipefail
TAG=${1:-run}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
timeout -k 10 300 python -u -m pytest tests/test_recon_gpu.py -m gpu -x -q -k brecq --timeout 120 --timeout-method thread > $OUT/pytest_gather_$TAG.log 2>&1 || { echo "tests failed"; tail -30 $OUT/pytest_gather_$TAG.log; exit 1; }
tail -1 $OUT/pytest_gather_$TAG.log
for on in 1 0; do
  SSQ_BRECQ_GATHER_ONCE=$on timeout -k 10 600 python main_imagenet.py --arch resnet18 --n_bits_w 2 --n_bits_a 4 --weight 1.0 --bias_cal True --bias_ch_quant True > $OUT/e2e_gather${on}_$TAG.log 2>&1 || { echo "e2e failed"; tail -20 $OUT/e2e_gather${on}_$TAG.log; exit 1; }
  echo "GATHER_ONCE=$on: $(grep 'calibration finished' $OUT/e2e_gather${on}_$TAG.log | cut -c1-90)"
done
if [ "$(grep 'calibration finished' $OUT/e2e_gather1_$TAG.log | sed 's/.*block rec losses//')" == "$(grep 'calibration finished' $OUT/e2e_gather0_$TAG.log | sed 's/.*block rec losses//')" ]; then echo "block losses identical"; else echo "block losses DIFFER"; fi
bash $R/tools/act_anatomy.sh gather_$TAG
