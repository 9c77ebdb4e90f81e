"""Fused shifted-scale reconstruction (reference: quant/layer_recon_fused_shiftedScale.py).

block_recon_fused_shiftedScale learns the shift logits alpha of every ChannelQuant in a
block ('adaShift' mode: softmax mix of the per-shift floors + AdaRound soft round) against
the block's cached FP outputs:  loss = lp(p=2) + [count >= 0.2*iters] *
(lmdaR * sum(1-|2h(beta)-1|^b) + lmdaS * sum(1-|2p(alpha)-1|^b2)),  Adam(lr=1e-3).

Per iteration on the device: one gather launch, per conv one adaShift forward + MIOpen
conv, the fused loss+gradient kernel, conv backward, per conv the two-stage alpha-gradient
kernels with the shift regulariser folded in, and the optimizer step -- no host sync
(the reference syncs twice per iteration via .item()).  Values that the reference only
prints (the rounding regulariser on the never-optimised beta, the total loss) are
computed lazily when reported.  `bias_cal=True` additionally learns the output-channel
affine gamma^z/phi^z (QuantModule.alpha_out/beta_out), the README's --bias_cal flag.
"""
import numpy as np
import torch
from tqdm import tqdm

from .. import kernels as K
from ..parallel_dp import GradBucket, world
from ._engine import (BatchFeeder, IterationGraph, LazyValue, SsqAdam, as_float, backward_tail,
                      clear_stash, probe, run_backward, stash_block_weights)
from .quant_block import BaseQuantBlock
from .quant_layer import QuantModule

# A/B knob: deferred loss / epilogue finalizes inside the loop body (bit-identical either way)
DEFER_FINALIZE = True
# the iteration's prepared adaShift forward rides on its batch gather (K.deferred_prep_fwd)
FUSE_START = True
# world 1: the Adam step rides on the alpha backward's launch (SsqAdam.arm, ssq_adam_arm)
FUSE_ADAM = True
# A/B knob: the block's final epilogue + loss + its backward as one pass (bit-identical)
FUSE_TAIL = True


def print_ratio(quantizers):
    """layer_recon_fused_shiftedScale.py:13-21: histogram of the selected shift index."""
    for qt in quantizers:
        soft_target = qt.get_sig_soft_targets().detach().cpu().numpy()
        max_index = np.argmax(soft_target, axis=-1)
        values, counts = np.unique(max_index, return_counts=True)
        total_cnt = np.sum(counts)
        dump_str = ' '.join([f'{k}:{v:.3f}' for k, v in zip(values, counts / total_cnt)])
        print(f'{qt.name}[{total_cnt}] : {dump_str}')


def _weight_quantizers(module):
    mods = [module] if isinstance(module, QuantModule) else \
        [m for m in module.modules() if isinstance(m, QuantModule)]
    return mods


GRAPH_WARMUP = 3     # eager iterations before the iteration body is captured


def _block_hard_flags(quantizers):
    """layer_recon_fused_shiftedScale.py:125-129: hard rounding AND hard shift choice."""
    for q in quantizers:
        q.hard_round = True
        q.hard_targets = True
        q.shiftedDone = True


def _fused_loop(block, modules, iters, lmda, model, p, lr, bias_cal, batch_size, dp_average,
                verbose, iter_hook=None, graph=True, set_hard=_block_hard_flags):
    device = next(model.parameters()).device
    quantizers, opt_params, beta_rg = [], [], {}
    for m in modules:
        q = m.weight_quantizer
        q.init_v_beta(x=m.org_weight.data.clone().detach())
        opt_params += [q.alpha]
        quantizers += [q]
        # beta is not optimised here (the reference's opt_params line for it is commented
        # out, :65): its gradient is never read, so it is not computed.  The reference's
        # autograd would accumulate it into beta.grad; nothing observes that.
        beta_rg[q] = q.beta.requires_grad
        q.beta.requires_grad_(False)
        q.opt_mode = 'adaShift'
        # gamma^z / phi^z: learned only with --bias_cal (the reference's commented-out
        # opt_params lines :67-68); otherwise their gradient is not computed at all
        m.alpha_out.requires_grad_(bias_cal)
        m.beta_out.requires_grad_(bias_cal)
        if bias_cal:
            opt_params += [m.alpha_out, m.beta_out]
    on_gpu = opt_params[0].is_cuda
    use_graph = bool(graph and on_gpu and iters > GRAPH_WARMUP + 1)
    # one ssq_adam launch for all parameters; its per-step scalars ride on the index copy,
    # so the whole iteration can be replayed from a HIP graph
    optimizer = SsqAdam(opt_params, lr=lr) if on_gpu else torch.optim.Adam(opt_params, lr=lr)
    if verbose:
        print("number of elements in opt_params: {}".format(sum(t.numel() for t in opt_params)))
    loss_func = FusedScaleLossFunction(block, quantizers, round_loss='relaxation', lmda=lmda,
                                       max_count=iters, b_range=(20, 2), decay_start=0,
                                       warmup=0.2, p=p)
    # extra device words: [lambda_S, b2 | -lr/bc1, sqrt(bc2)] refreshed with every index copy
    feeder = BatchFeeder(torch.cat(block.cached_inp_features), torch.cat(block.cached_out_features),
                         batch_size, device, extra_words=2)
    bucket = GradBucket(opt_params, average=dp_average) if world() > 1 else None
    # device (lambda_S, b2) read by the adaShift backward; it rides on the index copy
    regp = loss_func.arm(device, regp=feeder.extra[0:2])
    hyper = feeder.extra[2:4]
    last = {}

    # the loss value and gamma^z/phi^z finalizes ride on the next backward launch
    # (csrc/fin_tasks.h).  With a bucket (world > 1) the backward kernels write alpha and
    # gamma^z / phi^z straight into their bucket slices (K.grads_into) instead of handing
    # them to autograd, whose in-place add would read a finalize still queued; the queued
    # ones are flushed at the end of the body, before the collective
    defer = DEFER_FINALIZE and on_gpu

    # the fused tail (K.epilogue_loss_bwd) needs the p = 2 loss (the reference's default)
    fuse_tail = FUSE_TAIL and on_gpu and float(p) == 2.0
    # world 1: Adam runs where the gradients are finalised (no launch of its own)
    fuse_adam = FUSE_ADAM and on_gpu and bucket is None

    def body_pre():
        """One iteration on the device up to its exchange step: gather -> forward -> fused
        loss+grad -> backward.  No host sync, no host-side state: graph-capturable."""
        into = bucket.into_map() if (bucket is not None and defer) else {}
        with K.grads_into(into), K.deferred_finalize(defer):
            _body_pre(into)

    def _body_pre(into):
        if defer and any(t.grad is not None and t.data_ptr() not in into for t in opt_params):
            # a deferred gamma/phi gradient is only final after the next backward launch:
            # AccumulateGrad must take it over, never add it into an existing .grad
            raise RuntimeError("deferred finalizes need every parameter's .grad unset")
        if fuse_adam:
            # the optimizer step runs inside the alpha backward's launch (SsqAdam.arm)
            optimizer.arm(hyper)
        # every conv's What (one table) and the batch gather in ONE launch
        with K.deferred_prep_fwd(on_gpu and FUSE_START):
            if on_gpu:
                stash_block_weights(quantizers)
            cur_inp, cur_out = feeder.gather_lazy()
        K.TAIL_LAZY[0] = block if fuse_tail else None
        try:
            quant_out = block(cur_inp)
        finally:
            K.TAIL_LAZY[0] = None
        clear_stash(quantizers)
        tail = getattr(quant_out, '_ssq_tail', None)
        relu_in = getattr(quant_out, '_ssq_relu_inputs', None)
        if tail is not None:
            # the block's final epilogue, the loss and the epilogue's backward in one pass;
            # autograd resumes at the epilogue's inputs
            rec, grads = loss_func.fused_tail(tail, quant_out, cur_out)
            backward_tail(tail, grads)
        elif relu_in:
            # the block ends in the fused epilogue's ReLU: the loss pass writes the gradient
            # at the ReLU's input and backward starts from the epilogue's inputs
            rec, g_pre = loss_func.loss_and_grad(quant_out, cur_out, relu_mask=True)
            run_backward(list(relu_in), [g_pre] * len(relu_in))
        else:
            rec, g_out = loss_func.loss_and_grad(quant_out, cur_out)
            run_backward([quant_out], [g_out])
        last['rec'] = rec

    def body_post():
        """After the (RCCL) bucket all-reduce: the fused Adam step."""
        if on_gpu:
            optimizer.step(hyper=hyper)
        else:
            optimizer.step()

    graph_obj, ws_cache = None, {}
    start_loss = 0.0
    t = tqdm(range(iters), desc='', dynamic_ncols=True, disable=not verbose)
    for i in t:
        probe(i, opt_params)
        if iter_hook is not None:
            iter_hook(i)
        # reference-identical CPU randperm draw + this iteration's (lambda_S, b2): one H2D copy
        feeder.stage(feeder.draw(), extra=loss_func.schedule_pair() +
                     (optimizer.next_hyper() if on_gpu else (0.0, 0.0)))
        if use_graph and i == GRAPH_WARMUP:
            if bucket is None or not bucket.active:
                optimizer.zero_grad(set_to_none=True)
            # world > 1: two graphs around the eager bucket all-reduce (IterationGraph)
            graph_obj = IterationGraph(body_pre, body_post, bucket, ws_cache)
        if graph_obj is not None:
            graph_obj.replay()
        else:
            optimizer.zero_grad()
            if bucket is not None:
                bucket.attach_()
            body_pre()
            if bucket is not None:
                bucket.allreduce_()
            body_post()
        loss_func.bookkeep(last['rec'])
        if i % 500 == 0 and verbose:
            start_loss = max(start_loss, as_float(loss_func.rec_loss))
            t.set_description(f"{start_loss:.6f} -> {as_float(loss_func.rec_loss):.6f} "
                              f"{loss_func.round_loss_val} ")
    probe(iters, opt_params)
    if graph_obj is not None:
        torch.cuda.current_stream().synchronize()
        for p_ in opt_params:       # detach the grads from the graph's private pool
            p_.grad = None if p_.grad is None else p_.grad.clone()
        graph_obj.release()
        del graph_obj
    loss_func.disarm()
    for q, rg in beta_rg.items():
        q.beta.requires_grad_(rg)
    if iter_hook is not None:
        iter_hook(iters)

    rec_loss_out = []
    cur_inp, cur_out = feeder.head(batch_size)
    optimizer.zero_grad()
    with torch.no_grad():
        quant_out = block(cur_inp)
        loss_func(quant_out, cur_out)
    if verbose:
        print(f"Soft Round : {start_loss:.6f} -> {as_float(loss_func.rec_loss):.6f} "
              f"{loss_func.round_loss_val}")
    rec_loss_out.append(as_float(loss_func.rec_loss))
    set_hard(quantizers)
    with torch.no_grad():
        quant_out = block(cur_inp)
        loss_func(quant_out, cur_out)
    if verbose:
        print(f"Hard Round : {start_loss:.6f} -> {as_float(loss_func.rec_loss):.6f} "
              f"{loss_func.round_loss_val}")
    rec_loss_out.append(as_float(loss_func.rec_loss))
    if verbose:
        print_ratio(quantizers)
    model.eval()
    return rec_loss_out


def block_recon_fused_shiftedScale(block: BaseQuantBlock, iters: int = 20000, lmda: list = [1., 1.],
                                   model=None, test_loader=None, act=False, adaround=False,
                                   useShiftedScale=True, bias_cal=False, batch_size=32,
                                   dp_average=False, verbose=True, iter_hook=None, graph=True):
    """layer_recon_fused_shiftedScale.py:23-141 -> [soft rec loss, hard rec loss].
    graph=True replays the iteration body from a HIP graph after GRAPH_WARMUP eager
    iterations (at world > 1 as two graphs around the bucket all-reduce); the arithmetic
    and the batch draws are unchanged."""
    if act:
        # the reference's act branch builds ChannelQuantAct and calls its init_v, which
        # crashes (channelQuantAct.py:126-134): no working semantics exist to reproduce
        raise NotImplementedError("block_recon_fused_shiftedScale(act=True) is broken in the reference")
    block.train()
    return _fused_loop(block, _weight_quantizers(block), iters, lmda, model, 2.0, 0.001, bias_cal,
                       batch_size, dp_average, verbose, iter_hook, graph)


def layer_recon_fused_shiftedScale(layer: QuantModule, iters: int = 20000, lmda: list = [1., 1.],
                                   model=None, test_loader=None, act=False, adaround=False,
                                   useShiftedScale=True, bias_cal=False, batch_size=32,
                                   dp_average=False, verbose=True, graph=True):
    """layer_recon_fused_shiftedScale.py:144-221.  The reference raises UnboundLocalError
    (`opt_params += ...` before assignment, :156); this implements its evident intent: the
    block loop on one layer with p = 1.0 (:165) and Adam's default lr, finished with the
    layer variant's own flags (:207-211): hard shift targets + shiftedDone; with adaround
    the hard flag lands on the LAYER (not its quantizer), so the final 'Hard Round'
    evaluation keeps the soft rounding h(beta) either way -- reproduced as written."""
    model.train()

    def set_hard(quantizers):
        if adaround:
            layer.hard_round = True
        else:
            for q in quantizers:
                q.hard_targets = True
                q.shiftedDone = True

    return _fused_loop(layer, [layer], iters, lmda, model, 1.0, 0.001, bias_cal, batch_size,
                       dp_average, verbose, None, graph, set_hard=set_hard)


class FusedScaleLossFunction:
    """layer_recon_fused_shiftedScale.py:223-309.

    __call__(pred, tgt) is the reference-equivalent entry point (total loss tensor with
    autograd through the reconstruction term and the shift regulariser).  The loops use
    arm() + fused(): the shift-regulariser gradient is folded into each quantizer's
    adaShift backward kernel and the rounding regulariser (on beta, which the loop never
    optimises) is evaluated only when reported."""

    def __init__(self, block, quantizer, round_loss: str = 'relaxation', lmda: list = [1., 1.],
                 max_count: int = 2000, b_range: tuple = (10, 2), decay_start: float = 0.0,
                 warmup: float = 0.0, p: float = 2.0, adaround: bool = False):
        self.block = block
        self.quantizer = quantizer
        self.round_loss = round_loss
        self.lmdaR = lmda[0]
        self.lmdaS = lmda[1]
        self.loss_start = max_count * warmup
        self.itr = max_count
        self.p = p
        self.total_loss = self.rec_loss = self.round_loss_val = self.b = 0
        self.temp_decay = FusedLinearTempDecayShift(max_count, rel_start_decay=warmup + (1 - warmup) * decay_start,
                                                    start_b=b_range[0], end_b=b_range[1])
        self.temp_decay_shift = FusedLinearTempDecayShift(max_count * 3 / 4,
                                                          rel_start_decay=warmup + (1 - warmup) * decay_start,
                                                          start_b=b_range[0], end_b=b_range[1])
        self.count = 0
        self._reg_vals = {}

    def _schedule(self):
        b = self.temp_decay(self.count)
        b2 = self.temp_decay_shift(self.count)
        active = not (self.count < self.loss_start or self.round_loss == 'none')
        if self.round_loss not in ('none', 'relaxation'):
            raise NotImplementedError
        return (b, b2) if active else (0, 0), active

    # ---------------------------------------------------------------- reference entry point
    def __call__(self, pred, tgt, grad=None):
        rec_loss = K.lp_loss(pred, tgt, self.p)
        (b, b2), active = self._schedule()
        total = rec_loss
        R = S = 0
        if active:
            for qt in self.quantizer:
                R = R + K.round_reg(qt.beta, self.lmdaR, b)
                S = S + K.shift_reg(qt.alpha, self.lmdaS, b2, 0)
            total = rec_loss + R + S
        self._record(rec_loss, R, S, total, b)
        self.count += 1
        return total

    # ---------------------------------------------------------------- fused fast path
    def arm(self, device, regp=None):
        """Give every quantizer's adaShift backward the shift regulariser, with
        (lambda_S, b2) read from a device pair refreshed before each iteration
        (lambda_S = 0 during warm-up): `regp` (e.g. the BatchFeeder's extra word, which
        rides on the index copy) or a pair of its own that upload_schedule() fills.
        Returns that device pair."""
        self._regp = torch.zeros(2, dtype=torch.float32, device=device) if regp is None else regp
        self._regp_host = [torch.zeros(2, dtype=torch.float32, pin_memory=torch.cuda.is_available())
                           for _ in range(4)]
        self._regp_done = [None] * 4
        self._regp_k = 0
        for qt in self.quantizer:
            rows = qt.alpha.numel() // qt.alpha.shape[-1]
            vals = torch.zeros(rows, device=qt.alpha.device)
            self._reg_vals[id(qt)] = vals
            qt._fused_reg = (0.0, 0.0, vals, self._regp)
        return self._regp

    def schedule_pair(self):
        """This iteration's (lambda_S, b2) for the armed backward ((0, 0) in warm-up)."""
        (b, b2), active = self._schedule()
        return (float(self.lmdaS), float(b2)) if active else (0.0, 0.0)

    def upload_schedule(self, regp=None):
        """H2D (non-blocking, pinned ring) of this iteration's (lambda_S, b2)."""
        regp = self._regp if regp is None else regp
        (b, b2), active = self._schedule()
        slot = self._regp_k % len(self._regp_host)
        if self._regp_done[slot] is not None:
            self._regp_done[slot].synchronize()
        h = self._regp_host[slot]
        h[0], h[1] = (float(self.lmdaS), float(b2)) if active else (0.0, 0.0)
        regp.copy_(h, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        self._regp_done[slot] = ev
        self._regp_k += 1

    def disarm(self):
        for qt in self.quantizer:
            qt._fused_reg = None

    def fused_tail(self, tail, pred, tgt):
        """loss_and_grad + the final epilogue's backward in one pass (K.epilogue_loss_bwd);
        returns (rec_loss, the epilogue's input gradients)."""
        grads = K.epilogue_loss_bwd(tail, tgt, K._lp_M(pred, "none"))
        return grads[0][0], grads

    def loss_and_grad(self, pred, tgt, relu_mask=False):
        """One ssq_lp_loss pass: the loss value AND d loss / d pred (device only) -- or,
        with relu_mask, d loss / d (ReLU input) when pred is a ReLU output.  The caller
        back-propagates it -- exactly what total_loss.backward() delivers there; the
        regulariser terms reach alpha through the armed adaShift backward, and beta is
        never optimised by this loop."""
        rec_loss, grad = K.lp_loss_and_grad(pred, tgt, self.p, relu_mask=relu_mask)
        return rec_loss[0], grad

    def fused(self, pred, tgt):
        """loss_and_grad + the host bookkeeping of one iteration."""
        rec_loss, grad = self.loss_and_grad(pred, tgt)
        self.bookkeep(rec_loss)
        return rec_loss, grad

    def bookkeep(self, rec_loss):
        """Host side of one iteration: lazy report values and count += 1."""
        (b, b2), active = self._schedule()
        if active:
            quants, lR = list(self.quantizer), self.lmdaR
            vals = [self._reg_vals[id(q)] for q in quants]
            R = LazyValue(lambda: sum(float(K.round_reg_value(q.beta, lR, b).item()) for q in quants))
            S = LazyValue(lambda: sum(float(v.sum().item()) for v in vals))  # filled by backward
            total = LazyValue(lambda: as_float(rec_loss) + R.get() + S.get())
        else:
            R = S = 0
            total = rec_loss
        self._record(rec_loss, R, S, total, b)
        self.count += 1

    def _record(self, rec, R, S, total, b):
        self.rec_loss = LazyValue(rec.detach())
        self.total_loss = total if isinstance(total, LazyValue) else LazyValue(total.detach())
        self._R, self._S = R, S
        self.b = b

    @property
    def round_loss_val(self):
        return f'R:{as_float(self._lazy(self._R)):.3f} S:{as_float(self._lazy(self._S)):.3f}'

    @round_loss_val.setter
    def round_loss_val(self, v):
        self._R = self._S = 0

    @staticmethod
    def _lazy(v):
        if isinstance(v, torch.Tensor):
            return LazyValue(v.detach())
        return v

    def report(self):
        return 'Total loss:\t{:.6f} (rec:{:.6f}, round:{})\tb={:.2f}'.format(
            as_float(self.total_loss), as_float(self.rec_loss), self.round_loss_val, self.b)


class FusedLinearTempDecayShift:
    """layer_recon_fused_shiftedScale.py:382-399."""

    def __init__(self, t_max: int, rel_start_decay: float = 0.2, start_b: int = 10, end_b: int = 2):
        self.t_max = t_max
        self.start_decay = rel_start_decay * t_max
        self.start_b = start_b
        self.end_b = end_b

    def __call__(self, t):
        if t < self.start_decay:
            return self.start_b
        rel_t = (t - self.start_decay) / (self.t_max - self.start_decay) if self.t_max != 0 else 1
        return self.end_b + (self.start_b - self.end_b) * max(0.0, (1 - rel_t))
