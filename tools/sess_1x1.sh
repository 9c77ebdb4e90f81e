# r3: 1x1 stride-2 forwards as one batched GEMM (FWD_1X1_GEMM) on and off, in one session:
# bench.py's recon + validation lines (no q/dq-only changes), alternating.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
TAG=${1:-g1x1}
for v in 1 0 1 0; do
  SSQ_FWD_1X1_GEMM=$v timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 --warmup 5 > $OUT/b1x1_${TAG}_$v.log 2>&1 || { tail $OUT/b1x1_${TAG}_$v.log; exit 1; }
  python3 - "$OUT/b1x1_${TAG}_$v.log" $v <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["recon"]["iters_per_s"]
print(json.dumps({"fwd_1x1_gemm": sys.argv[2], "all_blocks": d["recon"]["resnet18_all_blocks_iters_per_s"],
                  "layer2.0": r["layer2.0"], "layer3.0": r["layer3.0"], "layer4.0": r["layer4.0"],
                  "val_img_s": d["validation"]["images_per_s"], "val_ms": d["validation"]["ms_per_batch"]}))
PY
done
