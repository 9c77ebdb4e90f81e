"""ChannelQuantAct (reference: quant/channelQuantAct.py).

Only opt_mode 'none' runs in the reference: per-tensor q/dq at delta*shiftedScale with a
[0, n-1] clamp and torch.round -- not round_ste, so no gradient reaches x
(channelQuantAct.py:56-67) -> ssq_fq_fwd / ssq_fq_round_bwd here.  Its init_v refers to an
undefined `x` and a missing `isFC`/`x_q` (channelQuantAct.py:125-134, AttributeError /
NameError [probed]), and the 'adaShift' / 'adaround' branches read attributes that are
never created, so those modes raise here too, with an explicit message.
"""
import torch
from torch import nn
import torch.nn.functional as F

from .. import kernels as K
from .quant_layer import UniformAffineQuantizer


class ChannelQuantAct(nn.Module):
    @torch.no_grad()
    def __init__(self, uaq: UniformAffineQuantizer, shiftTarget: list = [2 / 2, 2 / 2]):
        super().__init__()
        self.n_bits = uaq.n_bits
        self.sym = uaq.sym
        self.delta = uaq.delta
        self.zero_point = uaq.zero_point
        self.n_levels = uaq.n_levels
        self.device = 'cuda:0'
        self.shiftedScale = 1.0
        self.shiftTarget = shiftTarget
        self.opt_mode = 'none'
        self.hard_targets = False
        self.gamma, self.zeta = -0.1, 1.1
        self.alpha = None
        self.shiftedDone = False
        self.disable_act_quant = getattr(uaq, 'disable_act_quant', False)

    def forward(self, x):
        if self.opt_mode == 'none':
            # asymmetric [0, n-1] clamp whatever uaq.sym says (channelQuantAct.py:63)
            return K.round_quant(x, self.delta, self.zero_point, self.n_bits, False,
                                 scale=self.shiftedScale)
        raise NotImplementedError(
            f"ChannelQuantAct opt_mode={self.opt_mode!r} is broken in the reference "
            "(channelQuantAct.py:38-61,125-134 read attributes that are never set)")

    def get_sig_soft_targets(self):
        return torch.clamp(F.softmax(self.alpha, dim=-1) * (self.zeta - self.gamma) + self.gamma, 0, 1)

    def get_soft_targets(self):
        return torch.clamp(torch.sigmoid(self.alpha) * (self.zeta - self.gamma) + self.gamma, 0, 1)

    def inverse_softmax(self, x):
        x = (x - self.gamma) / (self.zeta - self.gamma)
        logits = torch.log(x)
        return logits - torch.mean(logits, dim=-1, keepdim=True)

    def init_v(self):
        raise NotImplementedError(
            "ChannelQuantAct.init_v uses an undefined input tensor in the reference "
            "(channelQuantAct.py:126-134); no working semantics to reproduce")
