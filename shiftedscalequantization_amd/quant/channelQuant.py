"""ChannelQuant: the shifted-scale weight quantizer (reference: quant/channelQuant.py).

Per output channel delta/zero_point (copied from a UniformAffineQuantizer), and per INPUT
channel (conv) / per element (Linear) a soft choice among `shiftTarget` scale multipliers
via softmax logits alpha, plus AdaRound soft rounding via beta.

Hot arithmetic runs in libssq.so:
  'adaShift'             -> ssq_adashift_fwd / ssq_adashift_bwd (K5/K6)
  'learned_hard_sigmoid' -> ssq_lhs_fwd / ssq_lhs_bwd            (K7)
  'adaround' / 'none'    -> ssq_adaround_* / ssq_fq_fwd           (K8 / K1)
  init_v, init_v_beta, get_delta, init_beta -> ssq_shift_init / ssq_get_delta / ssq_rect_init (K9)
The reference keeps S W-sized candidate tensors in self.x_q; here the kernels recompute the
candidates from the weight captured at init time, and `x_q` is materialised on access
only (API compatibility).
"""
import torch
from torch import nn
import torch.nn.functional as F

from .. import kernels as K
from .quant_layer import UniformAffineQuantizer


class ChannelQuant(nn.Module):
    @torch.no_grad()
    def __init__(self, delta, uaq: UniformAffineQuantizer, weight_tensor: torch.Tensor,
                 shiftTarget: list = [2 / 2, 2 / 2], act=False, name='--'):
        super().__init__()
        self.RUN_CHANNEL_WISE = True
        self.act = act
        self.n_bits = uaq.n_bits
        self.sym = uaq.sym
        self.delta = uaq.delta * delta                     # channelQuant.py:17
        self.zero_point = uaq.zero_point
        self.n_levels = uaq.n_levels
        self.device = weight_tensor.device
        self.isFC = len(self.delta.shape) != 4
        self.nchannel = (weight_tensor.shape[0], weight_tensor.shape[1])
        self.shiftedScale = 1.0
        self.shiftTarget = shiftTarget
        self.opt_mode = 'none'
        self.hard_targets = False
        self.hard_round = False
        self.gamma, self.zeta = -0.1, 1.1
        self.alpha = None
        self.beta = None
        self.deltaQuant = None
        self.shiftedDone = False
        self.name = name
        # state captured by init_v / init_v_beta: the candidates are recomputed from it
        self._src = None            # weight the candidates were built from
        self._src_delta = None      # delta at that time
        self._src_kind = None       # 'floor' (init_v_beta) | 'dequant' (init_v)
        self._xq_cache = None
        self._fused_reg = None      # (lambda, b, reg_vals) set by FusedScaleLossFunction
        self._prep = None           # (key, kernels.AdaShiftPrep) of the prepared path
        self._stash = None          # What computed ahead by the block's batched launch

    # ------------------------------------------------------------------ candidates
    @property
    def x_q(self):
        """The reference's list of S candidate tensors (channelQuant.py:27,208,286),
        materialised lazily from the captured weight (kernels never need it)."""
        if self._src is None:
            return []
        if self._xq_cache is None:
            out = []
            for st in self.shiftTarget:
                if self._src_kind == 'floor':
                    out.append(torch.floor(self._src / (self._src_delta * st)))
                else:
                    y, _ = K.fake_quant_fwd(self._src, self._src_delta, self.zero_point,
                                            self.n_bits, self.sym, scale=st, ste=False)
                    out.append(y)
            self._xq_cache = out
        return self._xq_cache

    @x_q.setter
    def x_q(self, v):
        self._xq_cache = list(v) if v else None

    # ------------------------------------------------------------------ forward
    def _prepared(self):
        """The prepared adaShift state (packed floors + h(beta), computed once) when the
        loop-invariant inputs allow it: conv weight, S <= 4, floor candidates, beta not
        being learned.  Rebuilt whenever beta, the hard_round flag or the captured weight
        change (key below); None -> the recomputing kernels.  A trainable beta is never
        prepared, also not under no_grad: an optimizer that writes it through raw pointers
        (SsqAdam) leaves beta._version unchanged, so the key could not see the update."""
        if (self.isFC or self._src_kind != 'floor' or self.beta is None
                or len(self.shiftTarget) > 4 or not self._src.is_cuda
                or self.beta.requires_grad):
            self._prep = None
            return None
        key = (self._src.data_ptr(), self._src_delta.data_ptr(), self.beta.data_ptr(),
               self.beta._version, bool(self.hard_round), tuple(self.shiftTarget))
        if self._prep is None or self._prep[0] != key:
            prep = K.AdaShiftPrep(self._src, self.beta, self._src_delta, self.shiftTarget,
                                  self.hard_round)
            self._prep = (key, prep if prep.ok else None)
        return self._prep[1]

    def forward(self, x):
        if self._stash is not None:
            # this iteration's What, computed with the other convs of the block in one
            # launch (_engine.stash_block_weights); consumed once
            w, self._stash = self._stash, None
            return w
        if self.opt_mode == 'adaShift':
            prep = self._prepared()
            if prep is not None:
                return K.adashift_prepared(self.alpha, prep, self._src_delta, self.zero_point,
                                           self.n_bits, self.sym, self.hard_targets,
                                           reg=self._fused_reg)
            return K.adashift(self.alpha, self.beta, self._src, self._src_delta, self.zero_point,
                              self.shiftTarget, self.n_bits, self.sym, self.hard_targets,
                              self.hard_round, reg=self._fused_reg)
        elif self.opt_mode == 'adaround':
            return K.adaround(self.beta, x, self.delta, self.zero_point, self.n_bits, self.sym,
                              self.hard_round, scale=self.shiftedScale)
        elif self.opt_mode == 'none':
            y, _ = K.fake_quant_fwd(x, self.delta, self.zero_point, self.n_bits, self.sym,
                                    scale=self.shiftedScale, ste=False)
            return y
        elif self.opt_mode in 'learned_hard_sigmoid':  # substring test, channelQuant.py:81
            return K.lhs(self.alpha, self._src, self._src_delta, self.zero_point, self.shiftTarget,
                         self.n_bits, self.sym, self.hard_targets)
        else:
            raise ValueError('opt_mode is not defined')

    def shifted_x_quant(self):
        """channelQuant.py:96-118 (API mirror over the materialised candidates)."""
        p = self.get_sig_soft_targets()
        if p.dim() == 2:
            p = p.unsqueeze(0)
        xq = self.x_q
        if self.hard_targets:
            max_index = torch.argmax(p, dim=-1)
            x_out = xq[0]
            for i in range(1, len(self.shiftTarget)):
                mask = max_index == i
                if not self.isFC:
                    mask = mask.unsqueeze(-1).unsqueeze(-1)
                x_out = torch.where(mask, xq[i], x_out)
            return x_out
        if self.isFC:
            x_out = xq[0] * p[:, :, 0]
            for i in range(1, len(self.shiftTarget)):
                x_out = x_out + xq[i] * p[:, :, i]
        else:
            p = p.unsqueeze(-1).unsqueeze(-1)
            x_out = xq[0] * p[:, :, 0, :, :]
            for i in range(1, len(self.shiftTarget)):
                x_out = x_out + xq[i] * p[:, :, i, :, :]
        return x_out

    def get_sig_soft_targets(self):
        return torch.clamp(F.softmax(self.alpha, dim=-1) * (self.zeta - self.gamma) + self.gamma, 0, 1)

    def get_soft_targets(self):
        return torch.clamp(torch.sigmoid(self.alpha) * (self.zeta - self.gamma) + self.gamma, 0, 1)

    def get_soft_round(self):
        return torch.clamp(torch.sigmoid(self.beta) * (self.zeta - self.gamma) + self.gamma, 0, 1)

    # ------------------------------------------------------------------ inits
    def _capture(self, x, kind):
        self._prep = None
        self._src = x.detach().contiguous()
        self._src_delta = self.delta.detach().contiguous()
        self._src_kind = kind
        self._xq_cache = None

    def init_alpha(self, x: torch.Tensor, clip=0.80, device='cuda'):
        """channelQuant.py:158-191 (clip forced to 0.33), against the captured candidates."""
        mode = 0 if self._src_kind == 'floor' else 1
        alpha, _, _ = K.shift_init(x, self._src_delta, self.shiftTarget, zp=self.zero_point,
                                   n_bits=self.n_bits, sym=self.sym, mode=mode)
        if not self.isFC and x.shape[1] == 1:
            alpha = alpha.view(1, -1)
        return alpha

    def inverse_softmax(self, x):
        """channelQuant.py:193-199."""
        x = (x - self.gamma) / (self.zeta - self.gamma)
        logits = torch.log(x)
        return logits - torch.mean(logits, dim=-1, keepdim=True)

    @torch.no_grad()
    def init_v(self, x: torch.Tensor):
        """channelQuant.py:201-213: dequantized candidates + alpha; mode ->
        'learned_hard_sigmoid'."""
        self._capture(x, 'dequant')
        self.shiftedScale = 1.0
        self.alpha = nn.Parameter(self.init_alpha(x, clip=(0.90 - 0.05 * len(self.shiftTarget)),
                                                  device=self.device))
        self.opt_mode = 'learned_hard_sigmoid'

    def get_delta(self):
        """channelQuant.py:221-237: delta * shiftTarget[argmax p] per (Co, Ci)."""
        base = self._src_delta if self._src_delta is not None else self.delta
        return K.get_delta(base, self.alpha, self.shiftTarget, tuple(self._weight_shape()))

    def _weight_shape(self):
        if self._src is not None:
            return self._src.shape
        return (self.nchannel[0], self.nchannel[1]) if self.isFC else (self.nchannel[0], self.nchannel[1], 1, 1)

    @torch.no_grad()
    def init_v_beta(self, x: torch.Tensor):
        """channelQuant.py:279-294: integer-floor candidates, alpha from init_alpha on the
        floors, beta from the selected delta.  (Re-running it on an initialised quantizer
        raises TypeError in the reference; here it re-initialises.)"""
        print(f"{self.name}, Optimal shift candidates: ", self.shiftTarget)
        self._capture(x, 'floor')
        self.shiftedScale = 1.0
        alpha, beta, _ = K.shift_init(x, self._src_delta, self.shiftTarget, mode=0)
        if not self.isFC and x.shape[1] == 1:
            alpha = alpha.view(1, -1)
        self.alpha = nn.Parameter(alpha)
        self.beta = nn.Parameter(beta)

    @torch.no_grad()
    def update_delta(self):
        self.delta = self.get_delta()

    @torch.no_grad()
    def init_beta(self, x: torch.Tensor):
        """channelQuant.py:300-307: beta from the current delta (no shift)."""
        self.beta = nn.Parameter(K.rect_init(x, self.delta))

    def hard_codes(self):
        """Integer codes of the finished (hard target, hard round) quantizer, for export."""
        y, codes = K.adashift_codes(self.alpha, self.beta, self._src, self._src_delta,
                                    self.zero_point, self.shiftTarget, self.n_bits, self.sym)
        return y, codes
