"""Data-parallel helpers for calibration over RCCL (torch.distributed backend 'nccl' is
RCCL on ROCm; xGMI between the GPUs of a node).

The reference's only exchange is a per-iteration all-reduce (SUM) of every optimised
parameter's gradient (block_recon.py:100-102, linklink).  Here all gradients of one
iteration are packed into ONE flat fp32 bucket and reduced with a single collective --
a latency-bound message of a few KB (shift logits) to ~19 MB (BRECQ AdaRound) per block.
"""
import torch
import torch.distributed as dist


def world():
    return dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1


def rank():
    return dist.get_rank() if dist.is_available() and dist.is_initialized() else 0


class GradBucket:
    """Flat all-reduce bucket over a fixed list of parameters.

    average=False reproduces the reference (sum of per-rank gradients); average=True
    divides by the world size (keeps the single-GPU loss scale)."""

    def __init__(self, params, average=False):
        self.params = [p for p in params if p.requires_grad]
        self.average = average
        n = sum(p.numel() for p in self.params)
        dev = self.params[0].device if self.params else torch.device("cpu")
        self.flat = torch.zeros(n, dtype=torch.float32, device=dev)

    def allreduce_(self):
        ws = world()
        if ws == 1 or not self.params:
            return
        off = 0
        views = []
        for p in self.params:
            n = p.numel()
            v = self.flat[off:off + n]
            if p.grad is None:
                v.zero_()
            else:
                v.copy_(p.grad.reshape(-1))
            views.append((p, v))
            off += n
        dist.all_reduce(self.flat, op=dist.ReduceOp.SUM)
        if self.average:
            self.flat.div_(ws)
        for p, v in views:
            if p.grad is None:
                p.grad = v.view_as(p).clone()
            else:
                p.grad.copy_(v.view_as(p))


def all_average_(t):
    ws = world()
    if ws > 1:
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        t.div_(ws)
    return t


def shard_rows(n, r=None, ws=None):
    """Contiguous shard [lo, hi) of n calibration samples for rank r of ws."""
    r = rank() if r is None else r
    ws = world() if ws is None else ws
    per = (n + ws - 1) // ws
    lo = min(n, r * per)
    return lo, min(n, lo + per)
