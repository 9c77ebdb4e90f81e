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


# Test hook: when set to a list, every GradBucket.allreduce_ appends (local, reduced) flat
# copies -- the per-rank gradient before the collective and the summed one after it.
RECORD = None
# Bench hook: when set to a list, every device bucket's collective appends (start, end,
# elements) -- HIP events recorded on the current stream around it (the collective, the
# current stream's wait on it, and the average's division), for its time per iteration.
TIMING = None


class GradBucket:
    """Flat all-reduce bucket over the optimised parameters.

    average=False reproduces the reference (sum of per-rank gradients); average=True
    divides by the world size (keeps the single-GPU loss scale).

    The parameters that actually receive a gradient are fixed at the first call (the
    iteration's graph is the same on every rank and every iteration); a parameter that
    gets none keeps grad=None, as in the reference, so Adam skips it there too.  From then
    on each such parameter's .grad IS its slice of the flat buffer: attach_() (called after
    zero_grad) zeroes the buffer and points the grads at the slices, backward accumulates
    into them in place, and the collective runs on the buffer with no copy in or out."""

    def __init__(self, params, average=False):
        self.params = [p for p in params if p.requires_grad]
        self.average = average
        self.live = None
        self.flat = None
        self.views = []

    def _build(self):
        self.live = [p for p in self.params if p.grad is not None]
        n = sum(p.numel() for p in self.live)
        dev = self.live[0].device if self.live else torch.device("cpu")
        self.flat = torch.zeros(n, dtype=torch.float32, device=dev)
        off = 0
        for p in self.live:
            self.views.append(self.flat[off:off + p.numel()].view_as(p))
            off += p.numel()

    def attach_(self):
        """Zero the bucket and make it the storage of every live gradient."""
        if self.live is None:
            return
        self.flat.zero_()
        for p, v in zip(self.live, self.views):
            p.grad = v

    def into_map(self):
        """{param.data_ptr(): its bucket slice} for the live parameters (K.grads_into): the
        backward kernels write those gradients straight into the bucket.  Empty before the
        bucket is built (the first iteration hands the gradients over through .grad)."""
        if self.live is None:
            return {}
        return {p.data_ptr(): v for p, v in zip(self.live, self.views)}

    @property
    def active(self):
        """True once the bucket is built at world > 1 (what a graph capture needs)."""
        return world() > 1 and self.live is not None

    def allreduce_(self):
        ws = world()
        if ws == 1 or not self.params:
            return
        if self.live is None:
            self._build()
        for p, v in zip(self.live, self.views):
            if p.grad is None:
                v.zero_()          # (cannot happen after the first call; kept defensive)
                p.grad = v
            elif p.grad.data_ptr() != v.data_ptr():
                v.copy_(p.grad)    # first iteration, or a loop that reset the grads
                p.grad = v
        self.reduce_()

    def reduce_(self):
        """The collective alone, on the attached bucket (between two graph replays)."""
        ws = world()
        if RECORD is not None:
            RECORD.append(["local", self.flat.detach().clone()])
        timed = TIMING is not None and self.flat.is_cuda
        if timed:
            e0 = torch.cuda.Event(enable_timing=True)
            e0.record()
        if self.flat.numel():
            dist.all_reduce(self.flat, op=dist.ReduceOp.SUM)
            if self.average:
                self.flat.div_(ws)
        if timed:
            e1 = torch.cuda.Event(enable_timing=True)
            e1.record()
            TIMING.append((e0, e1, self.flat.numel()))
        if RECORD is not None:
            RECORD[-1].append(self.flat.detach().clone())


def all_average_(t):
    ws = world()
    if ws > 1:
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        t.div_(ws)
    return t


def broadcast_(t, src=0):
    if world() > 1:
        dist.broadcast(t, src)
    return t


def all_sum_(t):
    if world() > 1:
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return t


def shard_rows(n, r=None, ws=None):
    """Contiguous shard [lo, hi) of n calibration samples for rank r of ws."""
    r = rank() if r is None else r
    ws = world() if ws is None else ws
    per = (n + ws - 1) // ws
    lo = min(n, r * per)
    return lo, min(n, lo + per)


def replicated(module):
    """True when every floating-point parameter and buffer of `module` is bit-identical on
    all ranks: per tensor an exact integer checksum of its fp32 bit patterns (and its
    element count), compared between the all-reduced MIN and MAX.  The data-parallel
    recon keeps the learned parameters replicated by construction; this checks it."""
    ws = world()
    tensors = [t for t in list(module.parameters()) + list(module.buffers())
               if t.is_floating_point() and t.numel() > 0]
    if ws == 1 or not tensors:
        return True
    dev = tensors[0].device
    sig = torch.stack([torch.stack([t.detach().float().contiguous().view(torch.int32)
                                    .to(torch.int64).sum(),
                                    torch.tensor(t.numel(), device=dev)])
                       for t in tensors]).to(dev)
    lo, hi = sig.clone(), sig.clone()
    dist.all_reduce(lo, op=dist.ReduceOp.MIN)
    dist.all_reduce(hi, op=dist.ReduceOp.MAX)
    return bool(torch.equal(lo, hi))
