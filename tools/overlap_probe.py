"""Does a conv's input gradient (MIOpen) overlap its weight gradient (K17) on two streams?
Device time of both in sequence on one stream vs forked onto two streams (HIP graph of
`reps` iterations, events on the capturing stream), ResNet-18 block shapes, batch 32,
reference-faithful (deterministic) MIOpen solvers.  usage: python tools/overlap_probe.py"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from shiftedscalequantization_amd import kernels as K  # noqa: E402

torch.backends.cudnn.deterministic = True
torch.backends.cudnn.benchmark = False
dev = torch.device("cuda:0")
SHAPES = {"layer1": (64, 64, 56, 1), "layer2": (128, 128, 28, 1), "layer3": (256, 256, 14, 1),
          "layer4": (512, 512, 7, 1)}


def graph_ms(fn, reps=10, rounds=5):
    fn()
    torch.cuda.synchronize()
    g, ws = torch.cuda.CUDAGraph(), {}
    with K.A.workspace_scope(ws):
        with torch.cuda.graph(g):
            for _ in range(reps):
                fn()
    g.replay()
    torch.cuda.synchronize()
    ts = []
    for _ in range(rounds):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        g.replay()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b) / reps)
    return sorted(ts)[len(ts) // 2]


out = {}
side = torch.cuda.Stream(dev)
for name, (ci, co, hw, st) in SHAPES.items():
    x = torch.randn(32, ci, hw, hw, device=dev)
    w = torch.randn(co, ci, 3, 3, device=dev) * 0.05
    g = torch.randn(32, co, hw, hw, device=dev)

    def dgrad():
        return torch.ops.aten.convolution_backward(g, x, w, None, [1, 1], [1, 1], [1, 1], False,
                                                   [0, 0], 1, (True, False, False))[0]

    def wgrad():
        return K.conv_wgrad(x, g, w.shape, 1, 1, 1)

    def seq():
        dgrad()
        wgrad()

    def par():
        cur = torch.cuda.current_stream()
        side.wait_stream(cur)
        with torch.cuda.stream(side):
            wgrad()
        dgrad()
        cur.wait_stream(side)

    out[name] = {"dgrad_ms": graph_ms(dgrad), "wgrad_ms": graph_ms(wgrad), "seq_ms": graph_ms(seq),
                 "two_streams_ms": graph_ms(par)}
    out[name] = {k: round(v, 4) for k, v in out[name].items()}
print(json.dumps(out))
