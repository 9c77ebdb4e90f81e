"""Does cudnn.benchmark change MIOpen's solver choice under cudnn.deterministic?  Recon
iters/s of ResNet-18 layer3.0 / layer4.0 under deterministic, deterministic + benchmark and
benchmark alone, and a bitwise repeat check of a 7x7 3x3 conv's forward / input gradient /
weight gradient under deterministic + benchmark (profiles/r2_det_solver_probe.log)."""
import json, os, sys, time
import torch
sys.path.insert(0, os.getcwd())
from shiftedscalequantization_amd.recon_bench import run_block
dev = torch.device("cuda")
cud = torch.backends.cudnn
res = {}
for mode in ("det", "det+bench", "bench"):
    cud.deterministic = mode.startswith("det")
    cud.benchmark = mode.endswith("bench")
    for b in ("layer3.0", "layer4.0"):
        r = run_block(dev, b, iters=100)
        res[f"{mode}:{b}"] = round(r["ips"], 1)
print(json.dumps(res))
# bitwise determinism of MIOpen wgrad/fwd/dgrad under det+bench
cud.deterministic, cud.benchmark = True, True
x = torch.randn(32, 512, 7, 7, device=dev, requires_grad=True)
w = torch.randn(512, 512, 3, 3, device=dev, requires_grad=True)
outs = []
for _ in range(3):
    x.grad = w.grad = None
    y = torch.nn.functional.conv2d(x, w, None, 1, 1)
    y.backward(torch.ones_like(y))
    outs.append((y.detach().clone(), x.grad.clone(), w.grad.clone()))
print("bitwise repeat (fwd, dgrad, wgrad):", [all(torch.equal(o[k], outs[0][k]) for o in outs) for k in range(3)])
