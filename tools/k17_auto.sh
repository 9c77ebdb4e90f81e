#!/bin/bash
# Unattended K17 round: assemble -> build -> CPU tests -> GPU parity + rates -> commit, or
# revert on any failure; then a full GPU session with its profiles committed.
cd /root/repo
L=gpurun_out/k17_auto.log
echo "start $(date)" > $L
FILES="shiftedscalequantization_amd/csrc/conv_wgrad.hip shiftedscalequantization_amd/kernels.py tests/test_kernels_gpu.py"
build() { python -c "from shiftedscalequantization_amd import build as B; B.build()" >> $L 2>&1; }
revert() { echo "REVERT: $1" >> $L; git checkout -- $FILES >> $L 2>&1; build; echo "reverted $(date)" >> $L; }
python3 tools/k17_assemble.py >> $L 2>&1 || { revert assemble; exit 1; }
build || { revert build; exit 1; }
(cd /tmp && hipcc -O3 --offload-arch=gfx950 -std=c++17 -ffp-contract=off -fhip-fp32-correctly-rounded-divide-sqrt --cuda-device-only -S /root/repo/shiftedscalequantization_amd/csrc/conv_wgrad.hip -o /tmp/wg.s 2>/dev/null; grep -E "^\s+\.(vgpr|sgpr)_(count|spill_count)|\.name:\s+_ZN3ssq12wgrad_stage1" /tmp/wg.s) >> $L 2>&1
timeout 900 python -m pytest tests -x -q -m "not gpu" >> $L 2>&1 || { revert cpu_tests; exit 1; }
rm -f gpurun_out/k17_t.log
/usr/local/graft/bin/gpurun --timeout 900 -- 'mkdir -p gpurun_out && timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_recon_gpu.py -q -x -k "conv_wgrad or dwconv or recon" --timeout 120 --timeout-method thread > gpurun_out/k17_t.log 2>&1; echo "pytest_rc=$?" >> gpurun_out/k17_t.log; timeout -k 10 200 python tools/wgrad_bench.py > gpurun_out/k17_wb.log 2>&1; timeout -k 10 300 python tools/recon_policy_ab.py layer1.0,layer4.0 > gpurun_out/k17_rp.log 2>&1; exit 0' >> $L 2>&1
tail -5 gpurun_out/k17_t.log >> $L 2>/dev/null; cat gpurun_out/k17_wb.log gpurun_out/k17_rp.log >> $L 2>/dev/null
if grep -q "pytest_rc=0" gpurun_out/k17_t.log 2>/dev/null; then
  cp gpurun_out/k17_wb.log profiles/r1_wgrad_bench_v3.log; cp gpurun_out/k17_rp.log profiles/r1_recon_policy_ab_v3.log
  git add $FILES tools/k17_auto.sh tools/k17_assemble.py profiles/r1_wgrad_bench_v3.log profiles/r1_recon_policy_ab_v3.log
  git commit -qm "K17 stage 1 rewritten: 64x64 wave tiles (2x2 MFMA accumulators), chunks of 64/128 consecutive output pixels staged by LDS-DMA into two LDS buffers, layout chosen by a cost model; the Python gate asks the planner; more K17 parity cases" >> $L 2>&1 && echo COMMITTED >> $L
else
  revert gpu_tests; exit 1
fi
echo "k17 done $(date)" >> $L
/usr/local/graft/bin/gpurun --timeout 1200 -- 'bash tools/gpu_session.sh r1e' >> $L 2>&1
if tail -1 gpurun_out/bench_r1e.log | python3 -c "import json,sys; json.loads(sys.stdin.read())" 2>/dev/null; then
  tail -1 gpurun_out/bench_r1e.log > profiles/r1_bench.json
  cp gpurun_out/prof_r1e/bench_kernel_stats.csv profiles/r1_bench_kernel_stats.csv 2>/dev/null
  cp gpurun_out/prof_r1e/bench_domain_stats.csv profiles/r1_bench_domain_stats.csv 2>/dev/null
  cp gpurun_out/iter_anatomy_r1e.txt profiles/r1_recon_iter_anatomy.txt 2>/dev/null
  cp gpurun_out/pytest_gpu_r1e.log profiles/r1_pytest_gpu.log 2>/dev/null
  git add profiles && git commit -qm "Round-1 profiles: GPU test log, bench line (q/dq roofline with HBM read/write ceilings, recon rates in both conv-solver modes), rocprofv3 kernel stats, recon iteration anatomy" >> $L 2>&1 && echo PROFILES_COMMITTED >> $L
fi
echo "all done $(date)" >> $L
