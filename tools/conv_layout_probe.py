"""Time the recon iteration's conv work (fwd + dgrad + wgrad) of ResNet-18 blocks in NCHW
vs channels_last (MIOpen picks NHWC kernels: no batched transposes), fp32, batch 32."""
import json
import torch
import torch.nn.functional as F

dev = torch.device("cuda")


def t(fn, reps=20):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e3


res = []
for (C, H, stride, Cin) in ((64, 56, 1, 64), (512, 7, 1, 512), (128, 28, 1, 128), (256, 14, 1, 256)):
    for layout in ("nchw", "nhwc"):
        mf = torch.channels_last if layout == "nhwc" else torch.contiguous_format
        x = torch.randn(32, Cin, H, H, device=dev).contiguous(memory_format=mf)
        w = (torch.randn(C, Cin, 3, 3, device=dev) * 0.05).contiguous(memory_format=mf).requires_grad_(True)
        x.requires_grad_(True)
        y = F.conv2d(x, w, None, stride, 1)
        g = torch.randn_like(y)
        fwd = t(lambda: F.conv2d(x, w, None, stride, 1))

        def bwd():
            yy = F.conv2d(x, w, None, stride, 1)
            torch.autograd.grad(yy, (x, w), g)
        fb = t(bwd)
        res.append({"C": C, "H": H, "layout": layout, "fwd_us": round(fwd, 1), "fwd_bwd_us": round(fb, 1)})
        print(json.dumps(res[-1]), flush=True)
