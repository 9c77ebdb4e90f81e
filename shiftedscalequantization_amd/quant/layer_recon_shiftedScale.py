"""Two-phase shifted-scale reconstruction (reference: quant/layer_recon_shiftedScale.py).

Phase 1 (adaround=False): ChannelQuant.init_v -> learn the shift logits alpha in
'learned_hard_sigmoid' mode (soft mix of the dequantized candidates, ssq_lhs_fwd/bwd)
with loss = lp(p=2) + lmda * entropy(p(alpha)) after warm-up.
Phase 2 (adaround=True): update_delta to the selected shifted delta, init_beta, learn beta
in 'adaround' mode (ssq_adaround_fwd/bwd) with loss = lp + lmda*sum(1-|2h(beta)-1|^b).
"""
import torch
from tqdm import tqdm

from .. import kernels as K
from ..parallel_dp import GradBucket, world
from ._engine import BatchFeeder, LazyValue, as_float, probe
from .quant_block import BaseQuantBlock
from .quant_layer import QuantModule, UniformAffineQuantizer


def _loop(block, opt_params, optimizer, scheduler, loss_func, iters, batch_size, device, verbose,
          dp_average=False):
    feeder = BatchFeeder(torch.cat(block.cached_inp_features), torch.cat(block.cached_out_features),
                         batch_size, device)
    bucket = GradBucket(opt_params, average=dp_average) if world() > 1 else None
    start_loss = 0.0
    t = tqdm(range(iters), desc='', dynamic_ncols=True, disable=not verbose)
    for i in t:
        probe(i, opt_params)
        cur_inp, cur_out = feeder.next()
        optimizer.zero_grad()
        if bucket is not None:
            bucket.attach_()
        quant_out = block(cur_inp)
        err = loss_func(quant_out, cur_out)
        err.backward()
        if bucket is not None:
            bucket.allreduce_()
        optimizer.step()
        if scheduler is not None:
            scheduler.step()
        if i % 500 == 0 and verbose:
            start_loss = max(start_loss, as_float(loss_func.rec_loss))
            t.set_description(f"{start_loss:.6f} -> {as_float(loss_func.rec_loss):.6f} "
                              f"{as_float(loss_func.round_loss_val):.3f} ")
    probe(iters, opt_params)
    return feeder, start_loss


def _final_eval(block, feeder, loss_func, batch_size, start_loss, set_hard, verbose):
    out = []
    cur_inp, cur_out = feeder.head(batch_size)
    with torch.no_grad():
        loss_func(block(cur_inp), cur_out)
    if verbose:
        print(f"Soft Round : {start_loss:.6f} -> {as_float(loss_func.rec_loss):.6f} "
              f"{as_float(loss_func.round_loss_val):.3f}")
    out.append(as_float(loss_func.rec_loss))
    set_hard()
    with torch.no_grad():
        loss_func(block(cur_inp), cur_out)
    if verbose:
        print(f"Hard Round : {start_loss:.6f} -> {as_float(loss_func.rec_loss):.6f} "
              f"{as_float(loss_func.round_loss_val):.3f}")
    out.append(as_float(loss_func.rec_loss))
    return out


def block_recon_shiftedScale(block: BaseQuantBlock, iters: int = 20000, lmda: float = 1., model=None,
                             test_loader=None, act=False, adaround=False, useShiftedScale=True,
                             batch_size=32, verbose=True):
    """layer_recon_shiftedScale.py:12-124 -> [soft, hard] rec loss."""
    block.train()
    device = next(model.parameters()).device
    scheduler = None
    opt_params = []
    if act:
        for name, module in block.named_modules():
            if isinstance(module, QuantModule):
                if module.act_quantizer.disable_act_quant:
                    continue
                opt_params += [module.act_quantizer.delta]
            elif isinstance(module, UniformAffineQuantizer):
                if module.disable_act_quant:
                    continue
                opt_params += [module.delta]
        optimizer = torch.optim.Adam(opt_params, lr=4e-4)
        scheduler = torch.optim.lr_scheduler.CosineAnnealingLR(optimizer, T_max=iters, eta_min=0.)
    else:
        for name, module in block.named_modules():
            if isinstance(module, QuantModule):
                q = module.weight_quantizer
                if adaround:
                    if q.opt_mode == 'learned_hard_sigmoid':
                        q.update_delta()
                    q.init_beta(x=module.org_weight.data.clone().detach())
                    q.opt_mode = 'adaround'
                    opt_params += [q.beta]
                else:
                    q.init_v(x=module.org_weight.data.clone().detach())
                    opt_params += [q.alpha]
        optimizer = torch.optim.Adam(opt_params)
        if verbose:
            print("number of elements in opt_params: {}".format(sum(p.numel() for p in opt_params)))
    loss_func = ScaleLossBlockFunction(block, round_loss='none' if act else 'relaxation', lmda=lmda,
                                       max_count=iters, b_range=(20, 2), decay_start=0, warmup=0.2,
                                       p=2.0, adaround=adaround)
    feeder, start_loss = _loop(block, opt_params, optimizer, scheduler, loss_func, iters, batch_size,
                               device, verbose)

    def set_hard():
        if act:
            return
        for name, module in block.named_modules():
            if isinstance(module, QuantModule):
                if adaround:
                    module.weight_quantizer.hard_round = True
                else:
                    module.weight_quantizer.hard_targets = True
                    module.weight_quantizer.shiftedDone = True

    res = _final_eval(block, feeder, loss_func, batch_size, start_loss, set_hard, verbose)
    model.eval()
    return res


def layer_recon_shiftedScale(layer: QuantModule, iters: int = 20000, lmda: float = 1., model=None,
                             test_loader=None, act=False, adaround=False, useShiftedScale=True,
                             batch_size=32, verbose=True):
    """layer_recon_shiftedScale.py:262-338 -> [soft, hard] rec loss.  Reference quirk kept:
    in the adaround phase the final 'hard' flag is set on the layer, not on its quantizer
    (:326), so the 'Hard Round' evaluation still rounds softly."""
    model.train()
    device = next(model.parameters()).device
    q = layer.weight_quantizer
    if adaround:
        if q.opt_mode == 'learned_hard_sigmoid':
            q.update_delta()
        q.init_beta(x=layer.org_weight.data.clone().detach())
        q.opt_mode = 'adaround'
        opt_params = [q.beta]
    else:
        q.init_v(x=layer.org_weight.data.clone().detach())
        opt_params = [q.alpha]
    optimizer = torch.optim.Adam(opt_params)
    loss_func = ScaleLossFunction(layer, round_loss='none' if act else 'relaxation', lmda=lmda,
                                  max_count=iters, b_range=(20, 2), decay_start=0, warmup=0.2, p=2.0,
                                  adaround=adaround)
    feeder, start_loss = _loop(layer, opt_params, optimizer, None, loss_func, iters, batch_size,
                               device, verbose)

    def set_hard():
        if adaround:
            layer.hard_round = True
        else:
            q.hard_targets = True
            q.shiftedDone = True

    res = _final_eval(layer, feeder, loss_func, batch_size, start_loss, set_hard, verbose)
    model.eval()
    return res


class _ScaleLossBase:
    def __init__(self, round_loss, lmda, max_count, b_range, decay_start, warmup, p, adaround):
        self.round_loss = round_loss
        self.lmda = lmda
        self.loss_start = max_count * warmup
        self.itr = max_count
        self.p = p
        self.total_loss = self.rec_loss = self.round_loss_val = self.b = 0
        self.temp_decay = LinearTempDecayShift(max_count, rel_start_decay=warmup + (1 - warmup) * decay_start,
                                               start_b=b_range[0], end_b=b_range[1])
        self.adaround = adaround
        self.count = 0

    def _quantizers(self):
        raise NotImplementedError

    def __call__(self, pred, tgt, grad=None):
        rec_loss = K.lp_loss(pred, tgt, self.p)
        b = self.temp_decay(self.count)
        if self.count < self.loss_start or self.round_loss == 'none':
            b = round_loss = 0
        elif self.round_loss == 'relaxation':
            round_loss = 0
            for q in self._quantizers():
                if self.adaround:
                    round_loss = round_loss + K.round_reg(q.beta, self.lmda, b)
                else:
                    round_loss = round_loss + K.shift_reg(q.alpha, self.lmda, 0.0, 1)
        else:
            raise NotImplementedError
        total_loss = rec_loss + round_loss
        self.total_loss = LazyValue(total_loss.detach())
        self.rec_loss = LazyValue(rec_loss.detach())
        self.round_loss_val = LazyValue(round_loss.detach()) if isinstance(round_loss, torch.Tensor) else round_loss
        self.b = b
        self.count += 1
        return total_loss

    def report(self):
        return 'Total loss:\t{:.6f} (rec:{:.6f}, round:{:.6f})\tb={:.2f}'.format(
            as_float(self.total_loss), as_float(self.rec_loss), as_float(self.round_loss_val), self.b)


class ScaleLossBlockFunction(_ScaleLossBase):
    """layer_recon_shiftedScale.py:340-412."""

    def __init__(self, block, round_loss='relaxation', lmda=1., max_count=2000, b_range=(10, 2),
                 decay_start=0.0, warmup=0.0, p=2.0, adaround=False):
        super().__init__(round_loss, lmda, max_count, b_range, decay_start, warmup, p, adaround)
        self.block = block

    def _quantizers(self):
        return [m.weight_quantizer for m in self.block.modules() if isinstance(m, QuantModule)]


class ScaleLossFunction(_ScaleLossBase):
    """layer_recon_shiftedScale.py:414-486."""

    def __init__(self, layer, round_loss='relaxation', lmda=1., max_count=2000, b_range=(10, 2),
                 decay_start=0.0, warmup=0.0, p=2.0, adaround=False):
        super().__init__(round_loss, lmda, max_count, b_range, decay_start, warmup, p, adaround)
        self.layer = layer

    def _quantizers(self):
        return [self.layer.weight_quantizer]


class LinearTempDecayShift:
    """layer_recon_shiftedScale.py:488-505."""

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
