"""AdaRoundQuantizer (reference: quant/adaptive_rounding.py, BRECQ).

'learned_hard_sigmoid': floor(x/delta) + h(alpha) (soft) or [alpha >= 0] (hard), clamp,
dequant -> ssq_adaround_fwd/bwd (K8); alpha init -> ssq_rect_init.
"""
import torch
from torch import nn

from .. import kernels as K
from .quant_layer import UniformAffineQuantizer


class AdaRoundQuantizer(nn.Module):
    def __init__(self, uaq: UniformAffineQuantizer, weight_tensor: torch.Tensor,
                 round_mode='learned_round_sigmoid'):
        super().__init__()
        self.n_bits = uaq.n_bits
        self.sym = uaq.sym
        self.delta = uaq.delta
        self.zero_point = uaq.zero_point
        self.n_levels = uaq.n_levels
        self.round_mode = round_mode
        self.alpha = None
        self.soft_targets = False
        self.gamma, self.zeta = -0.1, 1.1
        self.beta = 2 / 3
        self._fused_reg = None      # (lambda, b, reg_dev): the BRECQ loop's folded round loss
        self.init_alpha(x=weight_tensor.clone())

    def forward(self, x):
        if self.round_mode == 'nearest':
            y, _ = K.fake_quant_fwd(x, self.delta, self.zero_point, self.n_bits, False, ste=False)
            return y
        elif self.round_mode == 'nearest_ste':
            return K.fake_quant(x, self.delta, self.zero_point, self.n_bits, False)
        elif self.round_mode == 'stochastic':
            # research mode, not on the calibration path: eager PyTorch like the reference
            x_floor = torch.floor(x / self.delta)
            rest = (x / self.delta) - x_floor
            x_int = x_floor + torch.bernoulli(rest)
            x_quant = torch.clamp(x_int + self.zero_point, 0, self.n_levels - 1)
            return (x_quant - self.zero_point) * self.delta
        elif self.round_mode == 'learned_hard_sigmoid':
            stash = getattr(self, '_stash', None)
            if stash is not None and stash[0] is x:
                return stash[1]            # computed with the block's others (stash_adaround)
            # adaptive_rounding.py:64 clamps to [0, n_levels-1] regardless of sym
            return K.adaround(self.alpha, x, self.delta, self.zero_point, self.n_bits, False,
                              not self.soft_targets, reg=self._fused_reg)
        else:
            raise ValueError('Wrong rounding mode')

    def get_soft_targets(self):
        return torch.clamp(torch.sigmoid(self.alpha) * (self.zeta - self.gamma) + self.gamma, 0, 1)

    def init_alpha(self, x: torch.Tensor):
        if self.round_mode == 'learned_hard_sigmoid':
            self.alpha = nn.Parameter(K.rect_init(x, self.delta))
        else:
            raise NotImplementedError
