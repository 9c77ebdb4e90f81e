"""BRECQ block reconstruction (reference: quant/block_recon.py).

Weight phase: every QuantModule's quantizer becomes an AdaRoundQuantizer
('learned_hard_sigmoid', ssq_adaround_fwd/bwd) and its W-sized alpha is learned with
loss = lp(p) + weight * sum(1 - |2h(alpha)-1|^b).  Act phase: the activation deltas
(ssq_fq_fwd/bwd STE, LSQ-style) are learned with Adam(lr) + cosine schedule.
multi_gpu=True all-reduces (SUM, as the reference's link.allreduce) every optimised
gradient each iteration -- here as ONE flat RCCL bucket (parallel_dp.GradBucket); the
reference's call crashes because `link` is never imported (block_recon.py:2,102).
"""
import contextlib
import os

import torch

from .. import kernels as K
from ..parallel_dp import GradBucket, world
from ._engine import (GRAPH_REPLAYS, ITER_PROBE, BatchFeeder, IterationGraph, LazyValue,
                      CosineLR, SsqAdam, as_float, backward_tail, clear_stash, frozen_except,
                      probe, run_backward, stash_adaround)
from .adaptive_rounding import AdaRoundQuantizer
from .data_utils import save_grad_data, save_inp_oup_data
from .quant_block import BaseQuantBlock
from .quant_layer import QuantModule, StraightThrough, cached_convs, pinned_weights
from .quant_model import QuantModel


def block_reconstruction(model: QuantModel, block: BaseQuantBlock, cali_data: torch.Tensor,
                         batch_size: int = 32, iters: int = 20000, weight: float = 0.01,
                         opt_mode: str = 'mse', asym: bool = False, include_act_func: bool = True,
                         b_range: tuple = (20, 2), warmup: float = 0.0, act_quant: bool = False,
                         lr: float = 4e-5, p: float = 2.0, multi_gpu: bool = False,
                         eval: bool = False, dp_average: bool = False):
    """block_recon.py:10-116."""
    return _reconstruct(model, block, [m for m in block.modules() if isinstance(m, QuantModule)],
                        cali_data, batch_size, iters, weight, opt_mode, asym, include_act_func,
                        b_range, warmup, act_quant, lr, p, multi_gpu, eval, dp_average,
                        block_level=True)


GRAPH_WARMUP = 3     # eager iterations before the iteration body is captured
ITER_HOOK = None     # optional callable(i, iters) at the top of every device-loop iteration (tools)
# optional callable(i) before iteration i is issued -- once per chunk replay (i its first
# iteration) -- and (iters) after the last: unlike ITER_HOOK it keeps the chunked replays,
# so the loop timed through it is the production loop (recon_bench)
TIMING_HOOK = None
# A/B knobs of the device loop, bit-identical either way (tests/test_recon_gpu.py); the
# environment's SSQ_BRECQ_FAST=0 starts with all of them off (end-to-end A/B runs):
_FAST = os.environ.get("SSQ_BRECQ_FAST", "1") != "0"
# the loss / epilogue finalizes ride on the next backward launch (csrc/fin_tasks.h; world 1)
DEFER_FINALIZE = _FAST
# a block's final epilogue, the loss (p = 2 weight phase, 2.4 act phase) and the epilogue's
# backward in one pass (K.epilogue_loss_bwd)
FUSE_TAIL = _FAST
# act phase: every weight quantizer's W_hat computed once for the loop (the weights are
# frozen there; quant_layer.pinned_weights)
PIN_WEIGHTS = _FAST
# act phase: the convs that read the block input (conv1, the downsample) computed once for
# every cached sample; each iteration gathers its batch's rows (quant_layer.cached_convs)
CACHE_CONVS = _FAST and os.environ.get("SSQ_BRECQ_CACHE_CONVS", "1") != "0"
# a loop in which nothing learns (the act phase of a layer whose act quantizer is the
# disabled network output: no optimised parameter reaches its output) runs only the
# iterations whose loss is reported (every 500th, and the last); the others keep only the
# reference's randperm draw and schedule steps, so every printed value, the final state and
# the RNG stream are unchanged
SKIP_FROZEN = _FAST
# weight phase: the block's AdaRound forwards in one launch and their backwards in one
# (_engine.stash_adaround)
STASH_ADAROUND = _FAST
# act phase with CACHE_CONVS: the batch input (when still read) and the cached convs' rows
# gathered two sources per launch (_engine.BatchFeeder.gather_many)
GATHER_ONCE = _FAST and os.environ.get("SSQ_BRECQ_GATHER_ONCE", "1") != "0"
# world 1, after the warm-up: this many iterations per graph replay (ChunkGraph), staged by
# one H2D copy -- for loops whose iteration is cheaper on the GPU than on the host (the
# fc's 20000-iteration AdaRound loop); 1 = one iteration per replay
CHUNK_ITERS = int(os.environ.get("SSQ_BRECQ_CHUNK", "25")) if _FAST else 1
# act phase with CACHE_CONVS: the cached convs' rows and (identity residual) the batch input
# are not gathered -- the epilogue kernels read them in place by the batch indices
# (kernels.rows_view, ssq_epilogue_*_rows): no gather launch and no batch copy per iteration
ROWS_IN_PLACE = CACHE_CONVS and os.environ.get("SSQ_BRECQ_ROWS", "1") != "0"


def _input_convs(block, qmodules, x):
    """The QuantModules whose conv reads the block input x directly and runs through
    forward_raw (the fused-epilogue path), found by one probing forward, with the number of
    output elements per sample of each."""
    hits, per_sample = [], {}

    def pre(m, args):
        if args and isinstance(args[0], torch.Tensor) and args[0].data_ptr() == x.data_ptr() \
                and m.epilogue_fusable(args[0]):
            hits.append(m)

    def post(m, args, out):
        if m in hits and isinstance(out, torch.Tensor):
            per_sample[m] = out[0].numel()

    hs = [m.register_forward_pre_hook(pre) for m in qmodules]
    hs += [m.register_forward_hook(post) for m in qmodules]
    try:
        with torch.no_grad():
            block(x)
    finally:
        for h in hs:
            h.remove()
    return [(m, per_sample.get(m, 0)) for m in qmodules if m in hits]


# cached_convs holds every cached sample's raw output of each input conv (822 MB per
# ResNet-18 layer1 conv at 1024 samples): only when all of them fit in this fraction of
# the device's free memory; otherwise the loop runs those convs every iteration as before
CACHE_CONVS_MEM_FRAC = 0.5


def _reconstruct(model, block, qmodules, cali_data, batch_size, iters, weight, opt_mode, asym,
                 include_act_func, b_range, warmup, act_quant, lr, p, multi_gpu, eval, dp_average,
                 block_level, graph=True):
    if eval:
        iters = 0
    model.set_quant_state(False, False)
    block.set_quant_state(True, act_quant)
    round_mode = 'learned_hard_sigmoid'
    if not include_act_func:
        org_act_func = block.activation_function
        block.activation_function = StraightThrough()

    if not act_quant:
        for m in qmodules:
            m.weight_quantizer = AdaRoundQuantizer(uaq=m.weight_quantizer, round_mode=round_mode,
                                                   weight_tensor=m.org_weight.data)
            m.weight_quantizer.soft_targets = True
        opt_params = [m.weight_quantizer.alpha for m in qmodules]
    else:
        if block_level:   # block_recon.py:64-71
            opt_params = [block.act_quantizer.delta] + [
                m.act_quantizer.delta for m in qmodules if m.act_quantizer.delta is not None]
        else:             # layer_recon.py:61
            opt_params = [block.act_quantizer.delta]

    loss_func = LossFunction(block, round_loss='none' if act_quant else 'relaxation', weight=weight,
                             max_count=iters, rec_loss=opt_mode, b_range=b_range, decay_start=0,
                             warmup=warmup, p=p, quant_modules=qmodules)
    if iters > 0:
        cached_inps, cached_outs = save_inp_oup_data(model, block, cali_data, asym, act_quant,
                                                     batch_size)
        device = next(model.parameters()).device
        cached_grads = save_grad_data(model, block, cali_data, act_quant, batch_size=batch_size) \
            if opt_mode != 'mse' else None
        feeder = BatchFeeder(cached_inps, cached_outs, batch_size, device, extra_words=2)
        bucket = GradBucket(opt_params, average=dp_average) if (multi_gpu or world() > 1) else None
        if opt_mode == 'mse' and opt_params[0].is_cuda:
            with frozen_except(block, opt_params):
                _fast_loop(block, qmodules, opt_params, loss_func, feeder, bucket, iters, act_quant,
                           lr, p, graph)
        else:
            _eager_loop(opt_params, loss_func, feeder, bucket, cached_grads, block, iters, act_quant,
                        lr)
    for m in qmodules:
        if isinstance(m.weight_quantizer, AdaRoundQuantizer):
            m.weight_quantizer.soft_targets = False
    if not include_act_func:
        block.activation_function = org_act_func


def _eager_loop(opt_params, loss_func, feeder, bucket, cached_grads, block, iters, act_quant, lr):
    """The reference's loop (block_recon.py:90-105) as written, for the Fisher losses and
    host tensors."""
    if not act_quant:
        optimizer, scheduler = torch.optim.Adam(opt_params), None
    else:
        optimizer = torch.optim.Adam(opt_params, lr=lr)
        scheduler = torch.optim.lr_scheduler.CosineAnnealingLR(optimizer, T_max=max(iters, 1),
                                                               eta_min=0.)
    for i in range(iters):
        probe(i, opt_params)
        perm = feeder.draw()
        cur_inp, cur_out = feeder.next(perm)
        cur_grad = cached_grads[perm.to(cached_grads.device)] if cached_grads is not None else None
        optimizer.zero_grad()
        if bucket is not None:
            bucket.attach_()
        out_quant = block(cur_inp)
        err = loss_func(out_quant, cur_out, cur_grad)
        err.backward()
        if bucket is not None:
            bucket.allreduce_()
        optimizer.step()
        if scheduler:
            scheduler.step()
    probe(iters, opt_params)


# BRECQ's layer loop on a Linear layer (the network's last layer, 20000 iterations in the
# end-to-end flow), AdaRound weight phase at world 1: the whole iteration as the fused K19
# pair (kernels.fc_recon_iter) instead of gather / AdaRound / GEMM / loss / GEMM / AdaRound
# backward / Adam launches.  A/B knob: SSQ_FUSE_FC=0.
FUSE_FC = _FAST and os.environ.get("SSQ_FUSE_FC", "1") != "0"


def _fc_fused_body(layer, qmodules, act_quant, p, bucket, feeder, optimizer, last):
    """The fused fc iteration's body, or None when the loop is not one it covers: a
    Linear QuantModule alone, soft AdaRound with per-row delta, no activation, no act
    quantizer, no gamma^z / phi^z affine, p = 2, world 1, batch <= 64, C_in a multiple of 64
    up to 4096."""
    import torch.nn.functional as F
    if not (FUSE_FC and not act_quant and bucket is None and float(p) == 2.0
            and ITER_PROBE[0] is None      # a probe may rewrite V: W^ is carried over
            and len(qmodules) == 1 and qmodules[0] is layer and isinstance(layer, QuantModule)):
        return None
    m = layer
    q = m.weight_quantizer
    if not (m.fwd_func is F.linear and m.use_weight_quant and m.cache_features == 'none'
            and m.se_module is None and isinstance(m.activation_function, StraightThrough)
            and (not m.use_act_quant or m.disable_act_quant) and m._affine_is_identity()
            and isinstance(q, AdaRoundQuantizer) and q.round_mode == 'learned_hard_sigmoid'
            and q.soft_targets and getattr(q, '_stash', None) is None):
        return None
    w, v = m.weight, q.alpha
    if w.dim() != 2:
        return None
    Co, Ci = int(w.shape[0]), int(w.shape[1])
    if not (w.is_cuda and w.is_contiguous() and v.is_contiguous()
            and q.delta.numel() == Co and q.zero_point.numel() == Co
            and feeder.inp.dim() == 2 and feeder.inp.shape[1] == Ci
            and feeder.out.dim() == 2 and feeder.out.shape[1] == Co
            and 1 <= feeder.bs <= 64 and Ci % 64 == 0 and 64 <= Ci <= 4096
            and feeder.inp.data_ptr() % 16 == 0):
        return None
    if len(optimizer.params) != 1 or optimizer.params[0] is not v:
        return None
    st = optimizer.state[v]
    b1, b2 = optimizer.param_groups[0]["betas"]
    eps = optimizer.param_groups[0]["eps"]
    bias = m.bias if (m.bias is None or m.train_bias) else m.bias.detach()
    gbuf = torch.empty(feeder.bs, Co, device=w.device)
    gv = torch.zeros_like(v)        # V's gradient, for anyone reading .grad
    # W^ of the first iteration (every later one is written by the previous iteration)
    with torch.no_grad():
        what = K.adaround(v, w, q.delta, q.zero_point, q.n_bits, False, False).detach().clone()

    def body():
        src = feeder.chunk_dev[feeder.slot] if feeder.slot is not None else feeder._dev
        loss, _ = K.fc_recon_iter(feeder.inp, feeder.out, src, feeder.bs, w.detach(), v.data,
                                  what, q.delta, q.zero_point, q.n_bits, bias, st["exp_avg"],
                                  st["exp_avg_sq"], b1, b2, eps, g=gbuf, gv_out=gv)
        v.grad = gv
        last['rec'] = loss
        last['step'] = True
    return body


def _fast_loop(block, qmodules, opt_params, loss_func, feeder, bucket, iters, act_quant, lr, p,
               graph):
    """Same iteration, device only: one H2D copy (batch indices + this iteration's
    (lambda, b)), gather, forward, one fused lp_loss value+gradient pass (at the input of a
    final fused-epilogue ReLU), backward with the round loss's gradient folded into the
    AdaRound backward, fused Adam.  After GRAPH_WARMUP eager iterations the body is
    replayed from a HIP graph (at world > 1 as two graphs around the bucket all-reduce,
    _engine.IterationGraph).  The cosine LR schedule (_engine.CosineLR: torch's
    CosineAnnealingLR recursion, value for value) is copied into Adam's device lr.
    Launch savings (module knobs above, bit-identical on or off): deferred finalizes with the
    Adam step riding on them, the block's fused tail, and in the act phase pinned weights and
    the block-input convs precomputed for every cached sample."""
    if ITER_HOOK is not None:
        ITER_HOOK(-1, iters)
    use_graph = bool(graph and iters > GRAPH_WARMUP + 1)
    defer = DEFER_FINALIZE and bucket is None
    fuse_tail = FUSE_TAIL and isinstance(block, BaseQuantBlock)
    wq_params = {id(t) for m in qmodules for t in m.weight_quantizer.parameters()}
    pin = PIN_WEIGHTS and act_quant and not any(id(t) in wq_params for t in opt_params)
    stash_ada = STASH_ADAROUND and not act_quant and isinstance(block, BaseQuantBlock)
    if act_quant:
        optimizer = SsqAdam(opt_params, lr=lr)
        # the reference's cosine schedule (CosineAnnealingLR(T_max=iters, eta_min=0)), value
        # for value (_engine.CosineLR)
        scheduler = CosineLR(lr, max(iters, 1), 0.)
    else:
        optimizer, scheduler = SsqAdam(opt_params), None
    regp, hyper = feeder.extra[0:2], feeder.extra[2:4]
    ada = [m.weight_quantizer for m in qmodules if isinstance(m.weight_quantizer, AdaRoundQuantizer)]
    if not act_quant:
        for q in ada:
            q._fused_reg = (0.0, 0.0, regp)
    last = {}
    need_input = [True]     # False once cached_convs serves every reader of the block input
    conv_rows = []          # cached_convs' (all rows, batch buffer) pairs, gathered with the input
    rows_mode = [False, False]   # (cached rows read in place, the batch input as a row view)

    def body_pre():
        with K.deferred_finalize(defer):
            _body_pre()
            K.A.flush_row_stage()      # (no kernel took the iteration's stage: a copy)
            if bucket is None:
                # world 1: the step inside the deferral, so it rides on the last pending
                # finalizes (ssq_adam: one launch for both)
                _step()

    def _body_pre():
        if rows_mode[0]:
            cur_inp, cur_out = feeder.rows_lazy(need_input[0], rows_mode[1])
        elif conv_rows:
            cur_inp, cur_out = feeder.gather_many(conv_rows, input_needed=need_input[0])
        else:
            cur_inp, cur_out = feeder.gather_lazy(input_needed=need_input[0])
        if stash_ada:
            stash_adaround(qmodules)
        K.TAIL_LAZY[0] = block if fuse_tail else None
        try:
            out = block(cur_inp)
        finally:
            K.TAIL_LAZY[0] = None
            if stash_ada:
                clear_stash([m.weight_quantizer for m in qmodules])
        tail = getattr(out, '_ssq_tail', None)
        if tail is not None:
            # the block's final epilogue, the loss and the epilogue's backward in one pass;
            # autograd resumes at the epilogue's inputs
            grads = K.epilogue_loss_bwd(tail, cur_out, K._lp_M(out, "none"), p)
            y, _, gamma, phi, res, _, q = tail
            live = [y, gamma, phi] + ([q.delta, q.zero_point] if q is not None else [])
            live += [res.y, res.gamma, res.phi] if isinstance(res, K.LazyRes) else [res]
            last['rec'] = grads[0]
            last['step'] = any(t is not None and t.requires_grad for t in live)
            if last['step']:
                backward_tail(tail, grads)
            return
        relu_in = getattr(out, '_ssq_relu_inputs', None)
        if not out.requires_grad:
            # no optimised parameter reaches the output (e.g. the act delta of a layer whose
            # act quantizer is disabled): the reference's backward yields no gradient for it
            # and its Adam step skips it -- only the loss value remains
            last['rec'], _ = K.lp_loss_and_grad(out, cur_out, p, want_grad=False)
            last['step'] = False
            return
        if relu_in:
            rec, g = K.lp_loss_and_grad(out, cur_out, p, relu_mask=True)
            run_backward(list(relu_in), [g] * len(relu_in))
        else:
            rec, g = K.lp_loss_and_grad(out, cur_out, p)
            run_backward([out], [g])
        last['rec'] = rec
        last['step'] = True

    def _step():
        if last['step']:
            optimizer.step(hyper=hyper)

    def body_post():
        if bucket is not None:
            _step()

    fc_body = _fc_fused_body(block, qmodules, act_quant, p, bucket, feeder, optimizer, last)
    if fc_body is not None:
        body_pre = fc_body          # gather, forward, loss, backward and Adam: two launches

    ws_cache = {}
    with contextlib.ExitStack() as stack:
        if pin:
            stack.enter_context(pinned_weights(qmodules))
            if CACHE_CONVS and feeder.N % feeder.bs == 0:
                found = _input_convs(block, qmodules, feeder.cur_inp)
                need = sum(n for _, n in found) * feeder.N * 4
                free = torch.cuda.mem_get_info(feeder.inp.device)[0]
                convs = [m for m, _ in found] if need <= CACHE_CONVS_MEM_FRAC * free else []
                if convs:
                    mode = "rows" if ROWS_IN_PLACE else GATHER_ONCE
                    conv_rows[:] = stack.enter_context(cached_convs(
                        convs, feeder.cur_inp, feeder.inp, feeder.didx, gathered=mode))
                    if ROWS_IN_PLACE:
                        stack.enter_context(K.row_views())
                        rows_mode[0] = True
                    if ROWS_IN_PLACE or not GATHER_ONCE:
                        conv_rows.clear()
                    readers = block.input_readers() if isinstance(block, BaseQuantBlock) \
                        else [block]
                    need_input[0] = not (readers and all(m in convs for m in readers))
                    ident = block.identity_input_convs() if isinstance(block, BaseQuantBlock) \
                        else None
                    # an identity residual the only other reader: the input as a row view
                    rows_mode[1] = bool(ROWS_IN_PLACE and need_input[0] and ident
                                        and all(m in convs for m in ident))
        _run(iters, loss_func, feeder, optimizer, scheduler, use_graph,
             bucket, body_pre, body_post, last, opt_params, ada, ws_cache)


# tools: when CHUNK_PROBE[0] is not None, the loop's chunk graph is timed once right after
# its capture (ChunkGraph.probe: back-to-back replays, which repeat its iterations' device
# work on the same staged words -- the loop's results are then not the reference's; timing
# runs only) and the µs per iteration are left here
CHUNK_PROBE = [None]


class ChunkGraph:
    """`n` consecutive iterations of a world-1 loop captured in ONE HIP graph: the host draws
    the n iterations' batch permutations (the reference's torch.randperm on the CPU
    generator, in order), schedules and Adam step constants ahead, stages them with one H2D
    copy (BatchFeeder.stage_chunk) and replays once -- a loop whose iteration is a few
    microseconds of GPU work per launch (the fc's AdaRound layer loop: 9 small launches)
    is no longer paced by the host's per-iteration work.  Iteration k of the graph starts
    with ssq_gather_rows2_staged on slot k; the kernels, their order and their operands are
    the single-iteration graph's, so the results are the same bits
    (test_brecq_chunked_loop_bit_identical)."""

    def __init__(self, body, optimizer, feeder, n, ws_cache, last):
        self.n, self.recs = n, []
        g = torch.cuda.CUDAGraph()
        try:
            with K.A.workspace_scope(ws_cache):
                with torch.cuda.graph(g):
                    for k in range(n):
                        # autograd steals each iteration's gradient into .grad (none is
                        # accumulated across iterations, as the eager loop's zero_grad)
                        optimizer.zero_grad(set_to_none=True)
                        feeder.slot = k
                        body()
                        self.recs.append(last['rec'])
        finally:
            feeder.slot = None
            K.A.ROW_STAGE.clear()      # a stage queued by a capture that raised
        self.graph = g
        self.grads = [p.grad for p in optimizer.params]

    def replay(self):
        self.graph.replay()
        GRAPH_REPLAYS["chunk"] = GRAPH_REPLAYS.get("chunk", 0) + 1

    def probe(self, reps=20):
        """µs per iteration of back-to-back replays (GPU work and launch boundaries only)."""
        self.graph.replay()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            self.graph.replay()
        e1.record()
        e1.synchronize()
        return e0.elapsed_time(e1) * 1e3 / (reps * self.n)


def _run(iters, loss_func, feeder, optimizer, scheduler, use_graph, bucket, body_pre,
         body_post, last, opt_params, ada, ws_cache):
    graph_obj = None
    graph_last = {}
    chunk_obj = None
    grads_of = {}        # the .grad tensors of each graph (restored for the one replayed last)
    skip_ok = (SKIP_FROZEN and bucket is None and ITER_HOOK is None and
               ITER_PROBE[0] is None and not loss_func.track_values)
    chunk_ok = (use_graph and CHUNK_ITERS > 1 and bucket is None and ITER_HOOK is None and
                ITER_PROBE[0] is None and not loss_func.track_values)
    last_graph = [None]
    if chunk_ok:
        feeder.enable_chunks(CHUNK_ITERS)

    def body():
        body_pre()
        body_post()

    def run_chunk(n):
        """Iterations i .. i + n - 1 from the chunk graph (n == CHUNK_ITERS)."""
        nonlocal chunk_obj
        perms, extras, sched = [], [], []
        rnd = 0.0
        for k in range(n):
            b, lam, active = loss_func.schedule()
            perms.append(feeder.draw())
            extras.append((lam, float(b)) + optimizer.next_hyper())
            sched.append((b, loss_func.count))
            if k == 0 and active and loss_func.wants_value():
                # the round-loss value from alpha before this step (the chunk's first)
                rnd = loss_func.round_value(b)
            if scheduler is not None:
                optimizer.param_groups[0]['lr'] = scheduler.step()
        feeder.stage_chunk(perms, extras)
        if chunk_obj is None:
            chunk_obj = ChunkGraph(body, optimizer, feeder, n, ws_cache, last)
            if CHUNK_PROBE[0] is not None:
                CHUNK_PROBE[0] = chunk_obj.probe()
            grads_of['chunk'] = chunk_obj.grads
        chunk_obj.replay()
        last_graph[0] = 'chunk'
        for k, (b, count) in enumerate(sched):
            loss_func.record(chunk_obj.recs[k][0], rnd if k == 0 else 0.0, b, count=count)

    try:
        i = 0
        while i < iters:
            if TIMING_HOOK is not None:
                TIMING_HOOK(i)
            if chunk_ok and graph_obj is not None and last.get('step'):
                # the chunk never spans an iteration whose value is reported (count % 500)
                # except as its first
                r = (loss_func.count + 1) % 500
                n = min(CHUNK_ITERS, iters - i, 500 - r if r else 500)
                if n == CHUNK_ITERS:
                    run_chunk(n)
                    i += n
                    continue
            if ITER_HOOK is not None:
                ITER_HOOK(i, iters)
            probe(i, opt_params)
            b, lam, active = loss_func.schedule()
            perm = feeder.draw()
            hyp = optimizer.next_hyper()
            if (skip_ok and last.get('step') is False and loss_func.count % 500 != 0
                    and i != iters - 1):
                if scheduler is not None:
                    optimizer.param_groups[0]['lr'] = scheduler.step()
                i += 1
                continue
            feeder.stage(perm, extra=(lam, float(b)) + hyp)
            # the round-loss value (reporting only) from alpha before this step, as the
            # reference's forward computes it
            rnd = loss_func.round_value(b) if (active and loss_func.wants_value()) else 0.0
            if use_graph and i == GRAPH_WARMUP:
                if bucket is None or not bucket.active:
                    optimizer.zero_grad(set_to_none=True)
                # world > 1: two graphs around the eager bucket all-reduce (IterationGraph)
                graph_obj = IterationGraph(body_pre, body_post, bucket, ws_cache)
                grads_of['single'] = [p_.grad for p_ in opt_params]
                # the graph's own loss buffer and step flag (a chunk graph captured later
                # leaves `last` pointing at its last iteration's)
                graph_last = dict(last)
            if graph_obj is not None:
                last.update(graph_last)
                graph_obj.replay()
                last_graph[0] = 'single'
            else:
                optimizer.zero_grad()
                if bucket is not None:
                    bucket.attach_()
                body_pre()
                if bucket is not None and last['step']:
                    bucket.allreduce_()
                body_post()
            rec = last['rec'][0]
            loss_func.record(rec, rnd, b)
            if scheduler is not None:
                optimizer.param_groups[0]['lr'] = scheduler.step()
            i += 1
        if ITER_HOOK is not None:
            ITER_HOOK(iters, iters)
        if TIMING_HOOK is not None:
            TIMING_HOOK(iters)
        probe(iters, opt_params)
    finally:
        for q in ada:
            q._fused_reg = None
        if graph_obj is not None:
            torch.cuda.current_stream().synchronize()
            if last_graph[0] in grads_of:
                # the gradients the last replayed graph wrote
                for p_, g_ in zip(opt_params, grads_of[last_graph[0]]):
                    p_.grad = g_
            for p_ in opt_params:       # detach the grads from the graph's private pool
                p_.grad = None if p_.grad is None else p_.grad.clone()
            graph_obj.release()
            del graph_obj
            chunk_obj = None


class LossFunction:
    """block_recon.py:119-182 (count incremented BEFORE the schedule, unlike the fused
    loss).  The report line every 500 counts is the only host sync.  schedule() /
    round_value() / record() are the same steps split for the device-only loop."""

    def __init__(self, block, round_loss: str = 'relaxation', weight: float = 1., rec_loss: str = 'mse',
                 max_count: int = 2000, b_range: tuple = (10, 2), decay_start: float = 0.0,
                 warmup: float = 0.0, p: float = 2., quant_modules=None):
        self.block = block
        self.round_loss = round_loss
        self.weight = weight
        self.rec_loss = rec_loss
        self.loss_start = max_count * warmup
        self.p = p
        self.temp_decay = LinearTempDecay(max_count, rel_start_decay=warmup + (1 - warmup) * decay_start,
                                          start_b=b_range[0], end_b=b_range[1])
        self.count = 0
        self._qmodules = quant_modules
        self.last_total = None
        self.track_values = False   # True: round_value() every iteration (tests)

    def _modules(self):
        if self._qmodules is not None:
            return self._qmodules
        return [m for m in self.block.modules() if isinstance(m, QuantModule)]

    def schedule(self):
        """count += 1; (b, lambda_eff, round loss active) for this iteration."""
        self.count += 1
        b = self.temp_decay(self.count)
        if self.count < self.loss_start or self.round_loss == 'none':
            return 0, 0.0, False
        if self.round_loss != 'relaxation':
            raise NotImplementedError
        return b, float(self.weight), True

    def wants_value(self):
        return self.track_values or self.count % 500 == 0

    def round_value(self, b):
        total = 0
        for m in self._modules():
            total = total + K.round_reg_value(m.weight_quantizer.alpha, self.weight, b)
        return total

    def record(self, rec_loss, round_loss, b, count=None):
        """count: the iteration's own count when the host scheduled ahead (ChunkGraph)."""
        count = self.count if count is None else count
        # no tensor op when there is no round term (keeps the device loop launch-free)
        total_loss = rec_loss if isinstance(round_loss, (int, float)) and round_loss == 0 \
            else rec_loss + round_loss
        self.last_total = LazyValue(total_loss.detach() if isinstance(total_loss, torch.Tensor)
                                    else total_loss)
        if count % 500 == 0:
            print('Total loss:\t{:.3f} (rec:{:.3f}, round:{:.3f})\tb={:.2f}\tcount={}'.format(
                float(total_loss), float(rec_loss), float(round_loss), b, count))
        return total_loss

    def __call__(self, pred, tgt, grad=None):
        b, _, active = self.schedule()
        if self.rec_loss == 'mse':
            rec_loss = K.lp_loss(pred, tgt, self.p)
        elif self.rec_loss == 'fisher_diag':
            rec_loss = ((pred - tgt).pow(2) * grad.pow(2)).sum(1).mean()
        elif self.rec_loss == 'fisher_full':
            a = (pred - tgt).abs()
            g = grad.abs()
            batch_dotprod = torch.sum(a * g, (1, 2, 3)).view(-1, 1, 1, 1)
            rec_loss = (batch_dotprod * a * g).mean() / 100
        else:
            raise ValueError('Not supported reconstruction loss function: {}'.format(self.rec_loss))
        round_loss = 0
        if active:
            for m in self._modules():
                round_loss = round_loss + K.round_reg(m.weight_quantizer.alpha, self.weight, b)
        return self.record(rec_loss, round_loss, b)


class LinearTempDecay:
    """block_recon.py:185-202."""

    def __init__(self, t_max: int, rel_start_decay: float = 0.2, start_b: int = 10, end_b: int = 2):
        self.t_max = t_max
        self.start_decay = rel_start_decay * t_max
        self.start_b = start_b
        self.end_b = end_b

    def __call__(self, t):
        if t < self.start_decay:
            return self.start_b
        rel_t = (t - self.start_decay) / (self.t_max - self.start_decay)
        return self.end_b + (self.start_b - self.end_b) * max(0.0, (1 - rel_t))
