"""Shared machinery of the reconstruction loops.

BatchFeeder: the loop's `cached[torch.randperm(N)[:batch]]` (layer_recon_fused_shiftedScale.py:
95-97) with the permutation drawn from the SAME torch CPU generator stream as the
reference, the indices staged through a ring of pinned host buffers (no host sync), and
both cached tensors gathered by one ssq_gather_rows2 launch into reused device buffers.

LazyValue: the reference calls .item() on the loss every iteration (a device->host sync,
layer_recon_fused_shiftedScale.py:296-298); here loss values stay on the device and are
read only when reported.
"""
import math

import numpy as np
import torch

from .. import kernels as K


class BatchFeeder:
    RING = 4
    # chunk capture with rows read in place: the iteration's words staged by its first K13
    # row-view forward (False: by a copy launch, as the gathering loops' _stage_only)
    STAGE_IN_K13 = True

    def __init__(self, cached_inp, cached_out, batch_size, device, extra_words=1):
        self.inp = cached_inp.to(device).contiguous()
        self.out = cached_out.to(device).contiguous()
        self.N = self.inp.shape[0]
        self.bs = min(batch_size, self.N)
        self.device = device
        pin = torch.cuda.is_available()
        # one pinned slot = the batch indices + one 8-byte word carrying two fp32 values
        # riding on the same H2D copy (the loop's (lambda_S, b2) schedule pair)
        self.ring = [torch.zeros(self.bs + extra_words, dtype=torch.int64, pin_memory=pin)
                     for _ in range(self.RING)]
        # numpy views of the pinned slots: the per-iteration host writes without torch ops
        self.ring_np = [r.numpy() for r in self.ring]
        self.done = [None] * self.RING
        self.k = 0
        self._dev = torch.zeros(self.bs + extra_words, dtype=torch.int64, device=device)
        self.extra_words = extra_words
        self.slot = None          # chunk capture: this iteration's row of chunk_dev
        self.chunk_dev = None
        self.didx = self._dev[:self.bs]
        self.extra = self._dev[self.bs:].view(torch.float32)      # 2*extra_words floats
        self.cur_inp = torch.empty((self.bs,) + tuple(self.inp.shape[1:]), device=device)
        self.cur_out = torch.empty((self.bs,) + tuple(self.out.shape[1:]), device=device)

    def draw(self):
        """One reference-identical draw: torch.randperm(N)[:batch_size] on the CPU."""
        return torch.randperm(self.N)[:self.bs]

    def _write_slot(self, hn, perm, extra):
        hn[:self.bs] = perm.numpy()
        if extra is not None:
            # float64 -> float32 round to nearest, as torch.as_tensor(extra, dtype=float32)
            hn[self.bs:].view(np.float32)[:len(extra)] = np.asarray(extra, dtype=np.float64)

    def enable_chunks(self, n):
        """Several iterations per graph replay (quant/block_recon.py ChunkGraph): a device
        ring of n iterations' words (indices + the iteration's extra words), filled by one
        H2D copy per chunk from one of two pinned host buffers."""
        w = self.bs + self.extra_words
        pin = torch.cuda.is_available()
        self.chunk_dev = torch.zeros(n, w, dtype=torch.int64, device=self.device)
        self.chunk_host = [torch.zeros(n, w, dtype=torch.int64, pin_memory=pin) for _ in range(2)]
        self.chunk_np = [t.numpy() for t in self.chunk_host]
        self.chunk_done = [None, None]
        self.chunk_k = 0

    def stage_chunk(self, perms, extras):
        """The words of len(perms) consecutive iterations into chunk_dev (one H2D copy)."""
        j = self.chunk_k % 2
        if self.chunk_done[j] is not None:
            self.chunk_done[j].synchronize()
        hn = self.chunk_np[j]
        for k, (perm, extra) in enumerate(zip(perms, extras)):
            self._write_slot(hn[k], perm, extra)
        n = len(perms)
        self.chunk_dev[:n].copy_(self.chunk_host[j][:n], non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        self.chunk_done[j] = ev
        self.chunk_k += 1

    def _gather2(self, s0, s1, d0, d1, first):
        """One ssq_gather_rows2 launch by the static indices; the iteration's first one,
        inside a chunk capture, reads its slot of chunk_dev and copies the slot into the
        static words the iteration's later launches read (ssq_gather_rows2_staged)."""
        if first and self.slot is not None:
            K.gather_rows2_staged(s0, self.chunk_dev[self.slot], self.bs, self._dev, s1,
                                  out0=d0, out1=d1)
        else:
            K.gather_rows2(s0, self.didx, s1, out0=d0, out1=d1)

    def _stage_only(self):
        """Chunk capture, an iteration without a gather launch: the slot's words by copy."""
        if self.slot is not None:
            self._dev.copy_(self.chunk_dev[self.slot])

    def stage(self, perm, extra=None):
        """One host -> device copy of the batch indices (and, optionally, fp32 values into
        self.extra) into the static device buffer."""
        slot = self.k % self.RING
        if self.done[slot] is not None:
            self.done[slot].synchronize()
        h, hn = self.ring[slot], self.ring_np[slot]
        self._write_slot(hn, perm, extra)
        self._dev.copy_(h, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        self.done[slot] = ev
        self.k += 1

    def gather(self):
        """One ssq_gather_rows2 launch from the static indices into the static batch."""
        K.gather_rows2(self.inp, self.didx, self.out, out0=self.cur_inp, out1=self.cur_out)
        return self.cur_inp, self.cur_out

    def gather_lazy(self, input_needed=True):
        """The batch input gathered (the conv needs it contiguous); the batch target as a
        K.Rows view that the loss pass reads in place.  input_needed=False: every reader of
        the batch input serves it from elsewhere (quant_layer.cached_convs), so only the
        buffer's identity is handed on."""
        if input_needed:
            self._gather2(self.inp, None, self.cur_inp, None, True)
        else:
            self._stage_only()
        return self.cur_inp, K.Rows(self.out, self.didx)

    def gather_many(self, pairs, input_needed=True):
        """gather_lazy for a loop that also gathers other per-sample row sources (the
        precomputed block-input convs, quant_layer.cached_convs(gathered=True)) by the same
        indices: the batch input and those sources two per ssq_gather_rows2 launch."""
        srcs = ([(self.inp, self.cur_inp)] if input_needed else []) + list(pairs)
        if not srcs:
            self._stage_only()
        for k in range(0, len(srcs), 2):
            (s0, d0), (s1, d1) = srcs[k], srcs[k + 1] if k + 1 < len(srcs) else (None, None)
            self._gather2(s0, s1, d0, d1, k == 0)
        return self.cur_inp, K.Rows(self.out, self.didx)

    def rows_lazy(self, input_needed=True, input_view=False):
        """gather_lazy for a loop whose cached rows are read in place (kernels.rows_view):
        no gather of the cached convs' rows; the batch input is gathered only when it is
        needed and input_view is off, and with input_view it is handed on as a row view of
        the cached inputs (its only other reader is the tail's residual, which reads rows)."""
        if input_needed and not input_view:
            self._gather2(self.inp, None, self.cur_inp, None, True)
        elif self.slot is not None and not self.STAGE_IN_K13:
            self._stage_only()
        elif self.slot is not None:
            # chunk capture: the iteration's first K13 row-view forward copies the ring row
            # into the static words (ssq_epilogue_fwd_rows stage_*), reading its row maps from
            # the ring row; any other kernel call first performs it as a copy (_capi.fptr)
            K.A.ROW_STAGE[:] = [(self.chunk_dev[self.slot], self._dev)]
        if input_view:
            K.rows_view(self.cur_inp, self.inp, self.didx)
        return self.cur_inp, K.Rows(self.out, self.didx)

    def next(self, perm=None):
        self.stage(self.draw() if perm is None else perm)
        return self.gather()

    def head(self, n):
        """cached[:n] (the final soft/hard evaluation batch)."""
        return self.inp[:n], self.out[:n]


try:
    from torch.autograd.graph import _engine_run_backward
except ImportError:         # another torch: its public entry point
    _engine_run_backward = None


def run_backward(roots, grads):
    """torch.autograd.backward(roots, grads) for gradients the loop built to match their roots
    (shape, dtype and device checked here), handed straight to the autograd engine as
    torch.autograd.backward hands them after its own check.  That check (_make_grads)
    imports torch.fx's symbolic-shape module on its first call with a gradient tensor: 0.78 s
    in the flow's first shift loop (profiles/r5_e2e_setup_probe.txt); the reference's
    backward starts from a scalar loss and never pays it."""
    roots, grads = tuple(roots), tuple(grads)
    if len(roots) != len(grads):
        raise RuntimeError("run_backward: one gradient per root")
    for r, g in zip(roots, grads):
        if r.shape != g.shape or r.dtype != g.dtype or r.device != g.device:
            raise RuntimeError(f"run_backward: gradient {tuple(g.shape)} {g.dtype} {g.device} "
                               f"for a root {tuple(r.shape)} {r.dtype} {r.device}")
    if _engine_run_backward is None:
        torch.autograd.backward(roots, grads)
        return
    _engine_run_backward(roots, grads, False, False, (), allow_unreachable=True,
                         accumulate_grad=True)


def backward_tail(tail, grads):
    """Resume autograd at a fused tail's inputs: the conv output y and the residual through
    their graphs; gamma^z / phi^z / the act quantizer's delta and zero point are leaves here
    (or views of leaves), accumulated as autograd would."""
    y, bias, gamma, phi, res, relu, q = tail
    _, gy, gres, ggm, gph, gd, gz, grg, grph = grads
    roots, grs = [y], [gy]
    leaves = [(gamma, ggm), (phi, gph)]
    if isinstance(res, K.LazyRes):
        # the downsample's deferred epilogue: gres is dL/d(its conv output); its gamma^z /
        # phi^z are leaves like the block's own
        leaves += [(res.gamma, grg), (res.phi, grph)]
        res = res.y
    if gres is not None:
        roots.append(res)
        grs.append(gres)
    if q is not None:
        leaves += [(q.delta, gd), (q.zero_point, gz)]
    for t, g in leaves:
        if g is None:
            continue
        g = g.view(t.shape)
        if t.is_leaf:
            if t.grad is None:
                t.grad = g
            else:
                # g may be a deferred-finalize output (fin_tasks.h): make it final before
                # another kernel reads it
                K.flush_finalize(g.device)
                t.grad.add_(g)
        else:
            roots.append(t)
            grs.append(g)
    run_backward(roots, grs)


def stash_block_weights(quantizers):
    """The adaShift What of every prepared conv quantizer of a block in ONE launch (their
    alpha backward then runs as one two-launch reduction): they depend only on alpha,
    fixed for the iteration.  Each quantizer's next forward returns its stashed What.
    Quantizers that cannot use the prepared path (Linear, S > 4, int8 overflow, beta being
    learned) are left to compute their own.  Graph-capturable (device work only)."""
    groups = {}
    for q in quantizers:
        if q.opt_mode != 'adaShift':
            continue
        prep = q._prepared()
        if prep is None:
            continue
        key = (prep.S, bool(q.hard_targets), id(q._fused_reg[3]) if q._fused_reg else None)
        groups.setdefault(key, []).append((q, prep))
    for (S, hard_t, _), members in groups.items():
        qs = [q for q, _ in members]
        reg = qs[0]._fused_reg
        if reg is not None:
            reg = (reg[0], reg[1], [q._fused_reg[2] for q in qs], reg[3])
        entries = [(p, q._src_delta, q.zero_point, q.n_bits, q.sym) for q, p in members]
        outs = K.adashift_prepared_multi([q.alpha for q in qs], entries, hard_t, reg=reg)
        for q, w in zip(qs, outs):
            q._stash = w


def stash_adaround(modules):
    """The AdaRound W_hat of every module of a block in ONE launch (and their backward in
    one, AdaRoundMultiFn): BRECQ's weight phase learns only the rounding variables, and
    every weight's W_hat depends on its own alone.  Each quantizer's next forward on its
    module's weight returns the stashed W_hat.  Graph-capturable (device work only)."""
    qs = [m for m in modules if getattr(m.weight_quantizer, 'round_mode', None) == 'learned_hard_sigmoid'
          and m.use_weight_quant and m.weight.dim() == 4]
    if len(qs) < 2 or len(qs) > 8:
        return
    q0 = qs[0].weight_quantizer
    hard = not q0.soft_targets

    def reg_key(q):
        r = getattr(q, '_fused_reg', None)
        return None if r is None else (r[0], r[1], id(r[2]))

    if any((not m.weight_quantizer.soft_targets) != hard or
           reg_key(m.weight_quantizer) != reg_key(q0) for m in qs):
        return
    entries = [(m.weight, m.weight_quantizer.delta, m.weight_quantizer.zero_point,
                m.weight_quantizer.n_bits, False, 1.0) for m in qs]
    outs = K.adaround_multi([m.weight_quantizer.alpha for m in qs], entries, hard, reg=q0._fused_reg)
    for m, w in zip(qs, outs):
        m.weight_quantizer._stash = (m.weight, w)


def clear_stash(quantizers):
    for q in quantizers:
        if getattr(q, '_stash', None) is not None:
            q._stash = None


class LazyValue:
    """A device scalar (or a thunk producing one) read on demand."""

    def __init__(self, v):
        self._v = v

    def get(self):
        v = self._v() if callable(self._v) else self._v
        if isinstance(v, torch.Tensor):
            return float(v.detach().reshape(-1)[0].item()) if v.numel() == 1 else float(v.sum().item())
        return float(v)

    def __float__(self):
        return self.get()

    def __format__(self, spec):
        return format(self.get(), spec)

    def __str__(self):
        return str(self.get())

    def __lt__(self, o):
        return self.get() < float(o)

    def __gt__(self, o):
        return self.get() > float(o)


def as_float(v):
    return v.get() if isinstance(v, LazyValue) else float(v)


class SsqAdam:
    """torch.optim.Adam (default hyper-parameters, no weight decay / amsgrad) as one
    ssq_adam launch over all parameters, following the single-tensor update the reference
    runs.  The step count and the bias corrections live on the host; step(hyper=...)
    reads this step's (-lr/bc1, sqrt(bc2)) from a device pair instead, so a captured HIP
    graph replays with each iteration's values (next_hyper() advances the count)."""

    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8):
        self.params = [p for p in params]
        self.param_groups = [{"params": self.params, "lr": lr, "betas": betas, "eps": eps}]
        self.state = {p: {"exp_avg": torch.zeros_like(p, memory_format=torch.contiguous_format),
                          "exp_avg_sq": torch.zeros_like(p, memory_format=torch.contiguous_format)}
                      for p in self.params}
        self.t = 0

    def zero_grad(self, set_to_none=True):
        for p in self.params:
            if p.grad is not None:
                if set_to_none:
                    p.grad = None
                else:
                    p.grad.zero_()

    def next_hyper(self):
        """Advance the step count; (-lr/(1-b1^t), sqrt(1-b2^t)) as the reference computes
        them in double precision."""
        self.t += 1
        g = self.param_groups[0]
        b1, b2 = g["betas"]
        return -(g["lr"] / (1 - b1 ** self.t)), (1 - b2 ** self.t) ** 0.5

    def arm(self, hyper):
        """Arm this step inside the next prepared alpha backward (K.adam_arm): the update
        then runs where each gradient is finalised, no Adam launch of its own; step()
        launches it only if that did not happen.  World 1 only (at world > 1 the gradients
        are all-reduced between the backward and the step)."""
        g = self.param_groups[0]
        b1, b2 = g["betas"]
        K.adam_arm(self.params, [self.state[p]["exp_avg"] for p in self.params],
                   [self.state[p]["exp_avg_sq"] for p in self.params], b1, b2, g["eps"], hyper)
        self._armed = True

    def step(self, hyper=None):
        if getattr(self, "_armed", False):
            self._armed = False
            if K.adam_take(self.params[0].device):
                return
        live = [p for p in self.params if p.grad is not None]
        if not live:
            return
        g = self.param_groups[0]
        b1, b2 = g["betas"]
        if hyper is None:
            nss, bc2s = self.next_hyper()
        else:
            nss, bc2s = 0.0, 1.0
        K.adam_step(live, [p.grad for p in live], [self.state[p]["exp_avg"] for p in live],
                    [self.state[p]["exp_avg_sq"] for p in live], b1, b2, g["eps"], hyper=hyper,
                    neg_step_size=nss, bc2_sqrt=bc2s)


class CosineLR:
    """The lr sequence of torch.optim.lr_scheduler.CosineAnnealingLR(T_max, eta_min) as the
    reference's act phase steps it once per iteration (Brecq block_recon.py:56-58): the
    scheduler's chainable recursion (CosineAnnealingLR.get_lr, torch 2.10) with the same
    expressions in the same order, so every value is the same double
    (tests/test_host.py pins it against torch's scheduler).  It replaces a shadow
    torch.optim.Adam + scheduler: constructing the first torch optimizer of a process
    imports torch._dynamo (0.78 s in the ResNet-18 flow's first act phase,
    profiles/r5_e2e_setup_probe.txt), and each shadow step cost ~30 us of host time."""

    def __init__(self, lr, T_max, eta_min=0.0):
        self.base_lr = self.lr = lr
        self.T_max = T_max
        self.eta_min = eta_min
        self.last_epoch = 0        # after the scheduler's initial step
        self._step_count = 1

    def step(self):
        """One scheduler.step(); returns the new lr."""
        self._step_count += 1
        self.last_epoch += 1
        e, T, m = self.last_epoch, self.T_max, self.eta_min
        if self._step_count == 1 and e > 0:
            self.lr = m + (self.base_lr - m) * (1 + math.cos((e) * math.pi / T)) / 2
        elif (e - 1 - T) % (2 * T) == 0:
            self.lr = self.lr + (self.base_lr - m) * (1 - math.cos(math.pi / T)) / 2
        else:
            self.lr = ((1 + math.cos(math.pi * e / T)) / (1 + math.cos(math.pi * (e - 1) / T))
                       * (self.lr - m) + m)
        return self.lr


class frozen_except:
    """Context: every parameter of `module` that requires grad but is not in `keep` is
    frozen for the loop's duration.  The reference's autograd also computes (and
    accumulates) those gradients -- the FP conv weights under a UAQ weight quantizer, the
    weight quantizers' delta / zero_point, the act zero_points -- but nothing reads them."""

    def __init__(self, module, keep):
        ids = {id(p) for p in keep}
        self.frozen = [p for p in module.parameters() if p.requires_grad and id(p) not in ids]

    def __enter__(self):
        for p in self.frozen:
            p.requires_grad_(False)
        return self

    def __exit__(self, *exc):
        for p in self.frozen:
            p.requires_grad_(True)


# replays per form ("single" graph, "split" around the collective): test / report hook
GRAPH_REPLAYS = {"single": 0, "split": 0}

# Test probe of the reconstruction loops: when set, called as ITER_PROBE[0](i, opt_params)
# at the start of iteration i (before its batch is drawn) and once more with i = iters
# after the last one.  At that point every p.grad still holds iteration i-1's gradient
# (before its Adam step consumed it; a graph replay writes the same tensors), and an
# in-place write to a parameter is what iteration i computes from (teacher forcing).
ITER_PROBE = [None]


def probe(i, opt_params):
    if ITER_PROBE[0] is not None:
        ITER_PROBE[0](i, opt_params)


class IterationGraph:
    """HIP-graph replay of a reconstruction iteration split at its one exchange step.

    world == 1 (or no bucket): pre() + post() captured as one graph.  world > 1: the
    gradient all-reduce cannot run inside the graph (gloo goes through the host; RCCL's
    collective is issued by torch on its own stream), so the body is captured as two graphs
    around it -- pre = zero the flat bucket the live gradients are views of, gather,
    forward, fused loss + gradient, backward (accumulating in place into the bucket);
    post = the fused Adam step -- and each iteration replays pre, runs the bucket's
    collective eagerly, and replays post.  Same kernels, same order, same bits as the eager
    iteration; the per-iteration launch work is two graph launches and one collective."""

    def __init__(self, pre, post, bucket, ws_cache):
        self.bucket = bucket if (bucket is not None and bucket.active) else None
        self.graphs = []
        with K.A.workspace_scope(ws_cache):
            if self.bucket is None:
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g):
                    pre()
                    post()
                self.graphs = [g]
            else:
                self.bucket.attach_()            # grads = views of the bucket (host side)
                g1, g2 = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
                with torch.cuda.graph(g1):
                    self.bucket.flat.zero_()
                    pre()
                with torch.cuda.graph(g2, pool=g1.pool()):
                    post()
                self.graphs = [g1, g2]

    def replay(self):
        self.graphs[0].replay()
        if self.bucket is not None:
            self.bucket.reduce_()
            self.graphs[1].replay()
        GRAPH_REPLAYS["split" if self.bucket is not None else "single"] += 1

    def release(self):
        self.graphs = []
