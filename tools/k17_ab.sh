#!/bin/bash
cd $GRAFT_REPO_ROOT
timeout -k 10 200 python tools/wgrad_bench.py > gpurun_out/k17ab_160.log 2>&1 || exit 1
SSQ_K17_MAXLDS=81920 timeout -k 10 200 python tools/wgrad_bench.py > gpurun_out/k17ab_80.log 2>&1 || exit 1
SSQ_K17_MAXLDS=53000 timeout -k 10 200 python tools/wgrad_bench.py > gpurun_out/k17ab_52.log 2>&1 || exit 1
