"""Is a conv's output for one sample independent of the other samples in its batch (and of
its position there)?  For each shape: the conv of the whole cache in consecutive batches vs
the conv of randomly gathered batches, compared bit for bit (the premise of
quant_layer.cached_convs)."""
import json
import sys

import torch
import torch.nn.functional as F

torch.backends.cudnn.deterministic = bool(int(sys.argv[1])) if len(sys.argv) > 1 else True
dev = torch.device("cuda")
g = torch.Generator(device=dev).manual_seed(0)
cases = {"toy_conv1_16x16": (64, 16, 16, 16, 32, 3, 2, 1), "toy_ds_1x1": (64, 16, 16, 16, 32, 1, 2, 0),
         "r18_layer1_conv1": (256, 64, 56, 56, 64, 3, 1, 1), "r18_layer2_0_conv1": (256, 64, 56, 56, 128, 3, 2, 1),
         "r18_layer2_0_ds": (256, 64, 56, 56, 128, 1, 2, 0), "r18_layer3_0_conv1": (256, 128, 28, 28, 256, 3, 2, 1),
         "r18_layer4_0_conv1": (256, 256, 14, 14, 512, 3, 2, 1), "r18_layer4_1_conv1": (256, 512, 7, 7, 512, 3, 1, 1)}
res = {}
for name, (N, C, H, W, Co, k, st, pad) in cases.items():
    bs = 32 if N >= 64 else 8
    x = torch.randn(N, C, H, W, device=dev, generator=g).relu_()
    w = torch.randn(Co, C, k, k, device=dev, generator=g) * 0.05
    full = torch.cat([F.conv2d(x[i:i + bs], w, None, st, pad) for i in range(0, N, bs)])
    bad = 0
    for t in range(4):
        idx = torch.randperm(N, device=dev)[:bs]
        y = F.conv2d(x[idx].contiguous(), w, None, st, pad)
        bad += int((y.view(torch.int32) != full[idx].view(torch.int32)).any(dim=(1, 2, 3)).sum())
    res[name] = {"batch": bs, "samples_differing_of_%d" % (4 * bs): bad}
print(json.dumps({"deterministic": torch.backends.cudnn.deterministic, "cases": res}))
