"""UniformAffineQuantizer and QuantModule (reference: quant/quant_layer.py).

Same class names, constructor arguments, attributes and forward semantics as the
reference; the arithmetic runs in the HIP kernels of libssq.so:
  * UniformAffineQuantizer.forward        -> ssq_fq_fwd / ssq_fq_bwd (K1/K2)
  * UniformAffineQuantizer.init_quantization_scale -> ssq_scale_init (K3/K4; no per-channel
    Python loop, no .item() syncs)
  * lp_loss                               -> ssq_lp_loss (K11)
Feature caching keeps tensors on the device by default (the reference moves every batch
to the host with .cpu(); quant_layer.py:247,278) -- identical values, no PCIe round trip.
"""
import contextlib
import os
from typing import Union

import torch
import torch.nn as nn
import torch.nn.functional as F

from .. import kernels as K

# Frozen-weight cache of a validation pass (frozen_weight_cache): module -> (key, W_hat).
_FROZEN_W = None

# A QuantModule's epilogue with an act quantizer and no gamma^z / phi^z (BRECQ's act phase
# without --bias_cal) through the general epilogue (K.epilogue) rather than bias_act_quant.
# A/B knob: SSQ_EPI_NONAFFINE_Q=0.
EPI_NONAFFINE_Q = os.environ.get("SSQ_EPI_NONAFFINE_Q", "1") != "0"


@contextlib.contextmanager
def frozen_weight_cache():
    """Inside this context, under torch.no_grad, every QuantModule quantizes its weight once
    and reuses that W_hat for the rest of the context.  validate_model (common.py:152-221)
    runs the whole pass in it: no quantizer changes during inference, so each batch's
    forward is bit-identical to recomputing W_hat, without the per-batch weight q/dq
    launches.  The cache is keyed on the module, its weight quantizer object, the weight
    tensor (identity and version) and the quantizer's tensors and mode flags
    (_quantizer_state), and is dropped when the context exits.  Writes through raw pointers
    (SsqAdam, graph replays) bump no version: nothing may train inside the context."""
    global _FROZEN_W
    prev, _FROZEN_W = _FROZEN_W, {}
    try:
        yield
    finally:
        _FROZEN_W = prev


# Weights pinned for a loop in which no weight quantizer learns (pinned_weights):
# module -> W_hat.
_PINNED_W = None


@contextlib.contextmanager
def pinned_weights(modules):
    """Inside this context every QuantModule of `modules` that quantizes its weight uses the
    W_hat computed once on entry.  For a reconstruction loop whose optimised parameters do
    not reach any weight quantizer (BRECQ's act-delta phase, block_recon.py:62-73, after
    the weight phase has fixed the rounding): every iteration's weight q/dq is then the same
    computation on the same frozen inputs, so reusing its result is bit-identical and saves
    the per-iteration weight launches (also inside a captured HIP graph).  The caller
    guarantees that nothing the weight quantizers read changes inside the context."""
    global _PINNED_W
    prev = _PINNED_W
    pinned = {} if prev is None else dict(prev)
    with torch.no_grad():
        for m in modules:
            if m.use_weight_quant and m.cache_features == 'none':
                pinned[m] = m.weight_quantizer(m.weight)
    _PINNED_W = pinned
    try:
        yield
    finally:
        _PINNED_W = prev


# Frozen convolutions of a reconstruction loop (cached_convs): module -> (the loop's batch
# input data_ptr, its shape, the conv's raw outputs for every cached sample, the device
# batch indices, the batch output buffer, whether the caller gathers into it).
_CONV_CACHE = None


@contextlib.contextmanager
def cached_convs(modules, batch_input, source, idx, gathered=False):
    """Inside this context each QuantModule of `modules`, when its forward gets the loop's
    batch buffer `batch_input`, returns the rows idx of its raw conv output precomputed for
    every sample of `source` (the cached block inputs) instead of running the conv.  For a
    loop in which the conv's input and weight are frozen -- BRECQ's act phase
    (block_recon.py:62-73): the block input comes from the cache and the weights are pinned
    (pinned_weights) -- the batch conv computes exactly those rows.  They are precomputed in
    batches of the loop's own size, the same conv call on the same shapes, so the gathered
    rows are the loop's bits (test_brecq_loop_knobs_bit_identical).  The caller guarantees
    that the weights do not change inside the context.  gathered=True: the caller gathers
    the rows itself (the context yields each module's (all rows, batch buffer) pair, e.g. for
    one launch per iteration that also gathers the batch input) and forward only hands the
    batch buffer on.  gathered="rows": nothing gathers them -- forward hands the batch buffer
    on as a row view of (all rows, idx) (kernels.rows_view), which the epilogue kernels read
    in place; the caller holds a kernels.row_views() context."""
    global _CONV_CACHE
    prev = _CONV_CACHE
    cache = {} if prev is None else dict(prev)
    bs = batch_input.shape[0]
    with torch.no_grad():
        for m in modules:
            # one buffer for every sample's rows, written batch by batch (no list + cat: the
            # peak stays one copy of the cached outputs)
            first = m.forward_raw(source[:bs])[0]
            rows = torch.empty((source.shape[0],) + tuple(first.shape[1:]), dtype=first.dtype,
                               device=first.device)
            rows[:bs].copy_(first)
            for i in range(bs, source.shape[0], bs):
                rows[i:i + bs].copy_(m.forward_raw(source[i:i + bs])[0])
            cache[m] = (batch_input.data_ptr(), tuple(batch_input.shape), rows, idx,
                        torch.empty_like(first), gathered)
            del first
    _CONV_CACHE = cache
    try:
        yield [(cache[m][2], cache[m][4]) for m in modules]
    finally:
        _CONV_CACHE = prev


_STATE_FLAGS = ('soft_targets', 'hard_round', 'hard_targets', 'opt_mode', 'shiftedScale',
                'round_mode', 'n_bits')


def _quantizer_state(q):
    """What a weight quantizer's output depends on besides the weight: every tensor it holds
    (identity, storage, version counter) and its mode flags.  SsqAdam and graph replays write
    parameters through raw pointers without bumping _version, so the frozen-weight cache is
    only sound while nothing trains -- validate_model's pass (no_grad, no optimizer)."""
    ts = tuple((k, id(v), v.data_ptr(), v._version) for k, v in sorted(vars(q).items())
               if isinstance(v, torch.Tensor))
    ps = tuple((k, id(v), v.data_ptr(), v._version) for k, v in q.named_parameters(recurse=False))
    flags = tuple((k, getattr(q, k)) for k in _STATE_FLAGS if hasattr(q, k))
    return ts + ps + flags


class StraightThrough(nn.Module):
    """quant_layer.py:10-15."""

    def __init__(self, channel_num: int = 1):
        super().__init__()

    def forward(self, input):
        return input


def round_ste(x: torch.Tensor):
    """quant_layer.py:18-22 (API mirror; the q/dq kernels fold it in)."""
    return (x.round() - x).detach() + x


def lp_loss(pred, tgt, p=2.0, reduction='none'):
    """quant_layer.py:25-32: (pred-tgt).abs().pow(p).sum(1).mean() ('none') or .mean()."""
    return K.lp_loss(pred, tgt, p, reduction)


class UniformAffineQuantizer(nn.Module):
    """quant_layer.py:35-185.  Asymmetric/symmetric fake quantization, per tensor or per
    output channel; delta/zero_point initialised by 'max' or the 80-candidate 'mse' search."""

    def __init__(self, n_bits: int = 8, symmetric: bool = False, channel_wise: bool = False,
                 scale_method: str = 'max', leaf_param: bool = False, tune_delta_zero: bool = False,
                 ch: int = 64, disable_act_quant: bool = False):
        super().__init__()
        self.sym = symmetric
        assert 1 <= n_bits <= 8, 'bitwidth not supported'
        self.n_bits = n_bits
        self.n_levels = 2 ** self.n_bits
        self.delta = None
        self.zero_point = None
        self.raw_zero_point = None
        self.inited = False
        self.leaf_param = leaf_param
        self.channel_wise = channel_wise
        self.scale_method = scale_method
        self.disable_act_quant = disable_act_quant
        if not tune_delta_zero and not disable_act_quant:
            if leaf_param:
                self.delta = nn.Parameter(torch.tensor(0.0))
                self.zero_point = nn.Parameter(torch.tensor(0.0))
            elif type(ch) is int:
                self.delta = nn.Parameter(torch.zeros(size=(ch, 1)))
                self.zero_point = nn.Parameter(torch.zeros(size=(ch, 1)))
            elif len(ch) == 2:
                self.delta = nn.Parameter(torch.zeros(size=(ch[0], 1)))
                self.zero_point = nn.Parameter(torch.zeros(size=(ch[0], 1)))
            else:
                self.delta = nn.Parameter(torch.zeros(size=(ch[0], 1, 1, 1)))
                self.zero_point = nn.Parameter(torch.zeros(size=(ch[0], 1, 1, 1)))

    def forward(self, x: torch.Tensor):
        if self.inited is False:
            delta, zero_point, self.raw_zero_point = self.init_quantization_scale(x, self.channel_wise)
            self.delta = nn.Parameter(delta)
            self.zero_point = nn.Parameter(zero_point)
            self.inited = True
        return K.fake_quant(x, self.delta, self.zero_point, self.n_bits, self.sym)

    @torch.no_grad()
    def init_quantization_scale(self, x: torch.Tensor, channel_wise: bool = False):
        """quant_layer.py:100-166 on the device.  For per-tensor 'max' the reference returns
        a Python int zero point that nn.Parameter rejects (quant_layer.py:88,140); the
        evident intent (a 0-dim tensor) is implemented here."""
        d, z, r = K.scale_init(x, self.n_bits, self.sym, channel_wise, self.scale_method)
        return d.clone(), z.clone(), r.clone()

    def quantize(self, x, max, min):
        """quant_layer.py:168-175 (API mirror, used only for inspection)."""
        delta = (max - min) / (2 ** self.n_bits - 1)
        zero_point = (- min / delta).round()
        x_int = torch.round(x / delta)
        x_quant = torch.clamp(x_int + zero_point, 0, self.n_levels - 1)
        return (x_quant - zero_point) * delta

    def bitwidth_refactor(self, refactored_bit: int):
        assert 2 <= refactored_bit <= 8, 'bitwidth not supported'
        self.n_bits = refactored_bit
        self.n_levels = 2 ** self.n_bits

    def extra_repr(self):
        s = 'bit={n_bits}, scale_method={scale_method}, symmetric={sym}, channel_wise={channel_wise},' \
            ' leaf_param={leaf_param}'
        return s.format(**self.__dict__)


def fusable_act_quantizer(q, active):
    """The act quantizer `q` if its per-tensor q/dq can run inside the K13 epilogue pass
    (an initialised plain UniformAffineQuantizer with scalar delta/zp and no hooks), else
    None."""
    if not active or type(q) is not UniformAffineQuantizer or not q.inited:
        return None
    if q.delta is None or q.delta.numel() != 1 or q.zero_point.numel() != 1:
        return None
    if q._forward_hooks or q._forward_pre_hooks or not q.delta.is_cuda:
        return None
    return q


class QuantModule(nn.Module):
    """quant_layer.py:188-280: a Conv2d / Linear whose weight goes through
    `weight_quantizer` (any module: UAQ, ChannelQuant, AdaRoundQuantizer, ...), followed by
    the output-channel affine gamma^z=alpha_out / phi^z=beta_out, the activation and the
    activation quantizer.  The research-only greedy search methods (quant_layer.py:325-528)
    are out of scope."""

    def __init__(self, org_module: Union[nn.Conv2d, nn.Linear], weight_quant_params: dict = {},
                 act_quant_params: dict = {}, disable_act_quant: bool = False, se_module=None):
        super().__init__()
        if isinstance(org_module, nn.Conv2d):
            self.fwd_kwargs = dict(stride=org_module.stride, padding=org_module.padding,
                                   dilation=org_module.dilation, groups=org_module.groups)
            self.fwd_func = F.conv2d
        else:
            self.fwd_kwargs = dict()
            self.fwd_func = F.linear
        self.weight = org_module.weight
        self.org_weight = org_module.weight.data.clone()
        if org_module.bias is not None:
            self.bias = org_module.bias
            self.org_bias = org_module.bias.data.clone()
        else:
            self.bias = None
            self.org_bias = None
        self.use_weight_quant = False
        self.use_act_quant = False
        self.disable_act_quant = disable_act_quant
        weight_quant_params = dict(weight_quant_params)
        weight_quant_params['ch'] = self.weight.shape
        self.weight_quantizer = UniformAffineQuantizer(**weight_quant_params)
        act_quant_params = dict(act_quant_params)
        act_quant_params['disable_act_quant'] = disable_act_quant
        self.act_quantizer = UniformAffineQuantizer(**act_quant_params)

        self.activation_function = StraightThrough()
        self.ignore_reconstruction = False
        self.se_module = se_module
        self.extra_repr = org_module.extra_repr

        self.cache_features = 'none'
        self.cached_inp_features = []
        self.cached_out_features = []
        self.cache_to_host = False      # True: reference behaviour (.cpu() per batch)

        n_ch = self.weight.shape[0]
        if self.weight.dim() == 4:
            self.alpha_out = nn.Parameter(torch.ones(n_ch).view(1, n_ch, 1, 1))
            self.beta_out = nn.Parameter(torch.zeros(n_ch).view(1, n_ch, 1, 1))
        else:
            self.alpha_out = nn.Parameter(torch.ones(n_ch).view(1, n_ch))
            self.beta_out = nn.Parameter(torch.zeros(n_ch).view(1, n_ch))
        # gamma^z / phi^z are learned only with bias_cal: until then they need no grad
        self.alpha_out.requires_grad_(False)
        self.beta_out.requires_grad_(False)
        self._affine_key = None
        self._affine_identity = False
        self._affine_live = False
        self.train_bias = False
        self.selection = None
        self.selectionInited = False
        self.pathName = ''

    def _cache(self, t):
        t = t.detach()
        return t.cpu().clone() if self.cache_to_host else t.clone()

    def _apply(self, fn, *args, **kwargs):
        """.to() / .cuda() also move the FP copies org_weight / org_bias (plain tensor
        attributes, as in the reference, which leaves them behind on the old device)."""
        out = super()._apply(fn, *args, **kwargs)
        if isinstance(self.org_weight, torch.Tensor):
            self.org_weight = fn(self.org_weight)
        if isinstance(self.org_bias, torch.Tensor):
            self.org_bias = fn(self.org_bias)
        return out

    def _affine_is_identity(self):
        """True while gamma^z / phi^z are still their untouched initial (1, 0) tensors
        and nothing needs their gradient: then out*1+0 == out and the two passes (plus
        their backward) are skipped.  Once they have been trainable (--bias_cal) they
        count as live for good: the fused Adam and HIP-graph replays update them without
        bumping torch's version counter, so a version-keyed value check would go stale.
        Other in-place edits (torch ops) bump the version and trigger a re-check."""
        a, b = self.alpha_out, self.beta_out
        if a.requires_grad or b.requires_grad:
            self._affine_live = True
            return False
        if getattr(self, '_affine_live', False):
            return False
        key = (id(a), id(b), a._version, b._version, a.device)
        if key != self._affine_key:
            # first use on this device / after any change: check the values once
            self._affine_identity = bool(torch.all(a == 1).item() and torch.all(b == 0).item())
            self._affine_key = key
        return self._affine_identity

    def _weight_bias(self):
        if self.use_weight_quant and self.cache_features == 'none':
            if _PINNED_W is not None and self in _PINNED_W:
                weight = _PINNED_W[self]
            elif _FROZEN_W is not None and not torch.is_grad_enabled():
                key = (id(self.weight_quantizer), id(self.weight), self.weight._version,
                       _quantizer_state(self.weight_quantizer))
                hit = _FROZEN_W.get(self)
                if hit is None or hit[0] != key:
                    hit = (key, self.weight_quantizer(self.weight))
                    _FROZEN_W[self] = hit
                weight = hit[1]
            else:
                weight = self.weight_quantizer(self.weight)
            # no reconstruction ever optimises the conv bias: its gradient (a full
            # reduction over N,H,W per launch) is not requested
            bias = self.bias if (self.bias is None or self.train_bias) else self.bias.detach()
        else:
            weight = self.org_weight
            bias = self.org_bias
        return weight, bias

    def act_code(self):
        """The fused epilogues' activation code: 0 identity, 1 ReLU, 2 ReLU6."""
        if isinstance(self.activation_function, nn.ReLU6):
            return 2
        return 1 if isinstance(self.activation_function, nn.ReLU) else 0

    def epilogue_fusable(self, input):
        """The conv bias add, the gamma^z/phi^z affine and a ReLU / ReLU6 / identity
        activation can run as the fused K13 epilogue (bit-identical to the eager ops): a conv
        on the device, a constant bias, no SE module, no feature caching."""
        if not (input.is_cuda and self.fwd_func is F.conv2d and self.se_module is None
                and self.cache_features == 'none'
                and isinstance(self.activation_function, (nn.ReLU, nn.ReLU6, StraightThrough))):
            return False
        return not (self.bias is not None and self.bias.requires_grad and self.train_bias)

    def affine(self):
        """(gamma^z, phi^z) when the forward applies them (quant_layer.py:266-267), else
        (None, None)."""
        if self.use_weight_quant and self.cache_features == 'none' and not self._affine_is_identity():
            return self.alpha_out, self.beta_out
        return None, None

    def _conv(self, input, weight, bias=None):
        """The layer's conv / linear; a conv whose weight needs a gradient goes through
        K.conv2d (deterministic K17 weight gradient, see kernels.WGRAD_POLICY; a LazyEpi
        input folded into its im2col GEMM there)."""
        if self.fwd_func is F.conv2d and input.is_cuda and weight.requires_grad:
            out = K.conv2d(input, weight, **self.fwd_kwargs)
            return out if bias is None else out + bias.view(1, -1, 1, 1)
        return self.fwd_func(K.materialize_epi(input), weight, bias, **self.fwd_kwargs)

    def forward_raw(self, input):
        """(conv(input, W_hat) without bias, bias): for a parent block that fuses this
        module's bias add with its residual add and activation (see epilogue_fusable)."""
        weight, bias = self._weight_bias()
        if _CONV_CACHE is not None:
            hit = _CONV_CACHE.get(self)
            if hit is not None and hit[0] == input.data_ptr() and hit[1] == tuple(input.shape):
                if hit[5] == "rows":
                    return K.rows_view(hit[4], hit[2], hit[3]), bias
                if not hit[5]:
                    K.gather_rows2(hit[2], hit[3], out0=hit[4])
                return hit[4], bias
        return self._conv(input, weight), bias

    def forward(self, input: torch.Tensor):
        if self.cache_features == 'if':
            self.cached_inp_features += [self._cache(input)]
        act_q = self.use_act_quant and not self.disable_act_quant
        if self.epilogue_fusable(input):
            out, bias = self.forward_raw(input)
            relu = self.act_code()
            q = fusable_act_quantizer(self.act_quantizer, act_q)
            gamma, phi = self.affine()
            # (with an act quantizer only in the affine epilogue's form: the plain bias+act+q
            # pass has its own backward kernel, whose delta sums are not the affine one's)
            if (K.EPI_CONSUMER[0] is not None and (q is not None or not act_q)
                    and (q is None or gamma is not None)
                    and self.cache_features == 'none' and not self._forward_hooks):
                # the parent block's next conv folds this epilogue into its im2col GEMM
                # (kernels.EPI_CONSUMER); anything else materialises it
                return K.lazy_epilogue(out, bias, gamma, phi, relu, q)
            if gamma is not None or (q is not None and EPI_NONAFFINE_Q):
                # (no gamma^z / phi^z with an act quantizer: the general epilogue too, whose
                # backward sums the act delta per (n, c) row and hands its finalisation to
                # the next launch's task list -- bias_act_quant's backward finalises in a
                # launch of its own)
                out = K.epilogue(out, bias, gamma, phi, None, relu, q)
                act_q = act_q and q is None
            elif q is not None:
                out = K.bias_act_quant(out, bias, None, relu, q.delta, q.zero_point, q.n_bits,
                                       q.sym)
                act_q = False
            elif bias is not None or relu:
                out = K.bias_act(out, bias, None, relu)
            else:
                out = K.materialize(out)     # a row view leaves as the batch it stands for
        else:
            weight, bias = self._weight_bias()
            out = self._conv(input, weight, bias)
            if self.use_weight_quant and self.cache_features == 'none' and not self._affine_is_identity():
                out = out * self.alpha_out + self.beta_out
            if self.se_module is not None:
                out = self.se_module(out)
            out = self.activation_function(out)
        if act_q:
            out = self.act_quantizer(out)
        if self.cache_features == 'of':
            self.cached_out_features += [self._cache(out)]
        return out

    def set_quant_init_state(self):
        self.weight_quantizer.inited = True
        self.act_quantizer.inited = True

    def set_quant_state(self, weight_quant: bool = False, act_quant: bool = False):
        self.use_weight_quant = weight_quant
        self.use_act_quant = act_quant

    def disable_cache_features(self):
        self.cache_features = 'none'

    def clear_cached_features(self):
        self.cached_inp_features = []
        self.cached_out_features = []

    def getLoss(self, A, B, p=2.0):
        """quant_layer.py:319-323 (host-side report)."""
        loss = 0.0
        for i in range(len(B)):
            loss += lp_loss(A[i], B[i], p).detach()
        return float(loss)
