"""ChannelQuantMSE (reference: quant/channelQuantMSE.py): per-(Ci,kh,kw) input scale
chosen from `level` candidates by a code-range fit test, used by the shipped default
`ShiftedScaleQuant.py --test` path.  init_scale -> ssq_inpscale_search, forward ->
ssq_inpscale_fwd (K10)."""
import torch
from torch import nn

from .. import kernels as K
from .quant_layer import UniformAffineQuantizer


class ChannelQuantMSE(nn.Module):
    @torch.no_grad()
    def __init__(self, delta, uaq: UniformAffineQuantizer, weight_tensor: torch.Tensor,
                 shiftTarget: int = 2, act=False, opt_mode='max', level=1, threshold=1.0,
                 name='--'):
        super().__init__()
        self.RUN_CHANNEL_WISE = True
        self.act = act
        self.n_bits = uaq.n_bits
        self.sym = uaq.sym
        self.delta = uaq.delta * delta
        self.zero_point = uaq.zero_point
        self.n_levels = uaq.n_levels
        self.raw_zero_point = uaq.raw_zero_point
        self.device = weight_tensor.device
        self.isFC = len(self.delta.shape) != 4
        self.nchannel = (weight_tensor.shape[0], weight_tensor.shape[1])
        self.shiftTarget = shiftTarget
        self.x_q = []
        self.opt_mode = opt_mode
        self.hard_targets = False
        self.hard_round = False
        self.gamma, self.zeta = -0.1, 1.1
        self.alpha = None
        self.beta = None
        self.deltaQuant = None
        self.shiftedDone = False
        shape = (1, weight_tensor.shape[1]) if self.isFC else (1,) + tuple(weight_tensor.shape[1:])
        self.inp_scale = torch.ones(shape, device=self.device)
        self.scale_threshold = threshold
        self.scale_level = level
        self.name = name

    def mse_calc(self, x, x_quant, ignore_inp_scale=False):
        """channelQuantMSE.py:186-201 (host-side report)."""
        zero = torch.round(self.raw_zero_point / self.delta)
        x_float = (x_quant - zero) * self.delta * self.inp_scale if not ignore_inp_scale \
            else (x_quant - zero) * self.delta
        return torch.mean(torch.square(x_float - x)).item()

    @torch.no_grad()
    def init_scale(self, x):
        if self.opt_mode != 'max':
            raise NotImplementedError
        self.inp_scale = K.inpscale_search(x, self.delta, self.raw_zero_point, self.n_bits,
                                           self.scale_level, self.scale_threshold)

    def quant(self, x):
        zero_point = torch.round(self.raw_zero_point / self.delta)
        x_int = torch.round(x / self.inp_scale / self.delta) + zero_point
        return torch.clamp(x_int, 0, self.n_levels - 1)

    def forward(self, x):
        return K.inpscale_fwd(x, self.inp_scale, self.delta, self.raw_zero_point, self.n_bits)
