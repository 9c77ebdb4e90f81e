"""Quantized residual blocks (reference: quant/quant_block.py).

Branch structure, activation and block-level act quant after the element-wise add are
kept as in the reference.  setPathName is defined on BaseQuantBlock so every block type
works with QuantModel (the reference defines it only on QuantBasicBlock, so QuantModel
crashes on ResNet-50 / MobileNetV2 / RegNetX: quant_model.py:30 vs quant_block.py:119).
"""
import torch
import torch.nn as nn

from .. import kernels as K
from .. import nets
from .quant_layer import QuantModule, StraightThrough, UniformAffineQuantizer, fusable_act_quantizer


class BaseQuantBlock(nn.Module):
    def __init__(self, act_quant_params: dict = {}):
        super().__init__()
        self.use_weight_quant = False
        self.use_act_quant = False
        act_quant_params = dict(act_quant_params)
        act_quant_params['disable_act_quant'] = False
        self.act_quantizer = UniformAffineQuantizer(**act_quant_params)
        self.activation_function = StraightThrough()
        self.ignore_reconstruction = False
        self.cache_features = 'none'
        self.cached_inp_features = []
        self.cached_out_features = []
        self.cache_to_host = False
        self.selectionInited = False
        self.pathName = ''

    def set_quant_state(self, weight_quant: bool = False, act_quant: bool = False):
        self.use_weight_quant = weight_quant
        self.use_act_quant = act_quant
        for m in self.modules():
            if isinstance(m, QuantModule):
                m.set_quant_state(weight_quant, act_quant)

    def set_quant_init_state(self):
        for m in self.modules():
            if isinstance(m, QuantModule):
                m.set_quant_init_state()

    def set_quant_state_block(self, state, act=False):
        for m in self.modules():
            if isinstance(m, QuantModule):
                if act:
                    m.use_act_quant = state
                else:
                    m.use_weight_quant = state

    # the reference defines these twice; the second (block-level) definition wins
    def disable_cache_features(self):
        self.cache_features = 'none'

    def clear_cached_features(self):
        self.cached_inp_features = []
        self.cached_out_features = []

    def _cache(self, t):
        t = t.detach()
        return t.cpu().clone() if self.cache_to_host else t.clone()

    def setPathName(self, curName):
        self.pathName = curName
        for n, m in self.named_modules():
            if isinstance(m, QuantModule) and n:
                m.pathName = curName + '.' + n

    def _finish(self, out):
        out = self.activation_function(out)
        if self.use_act_quant:
            out = self.act_quantizer(out)
        return out

    def input_readers(self):
        """The QuantModules that read the block input and nothing else does (no identity
        residual), or None when the input is also used directly."""
        return None

    def identity_input_convs(self):
        """With an identity residual: the QuantModules that read the block input besides the
        residual add of the block's tail (_tail); None otherwise."""
        return None

    def _residual(self, ds, x):
        """ds(x), the downsample branch.  For the block the recon loop fuses (K.TAIL_LAZY)
        and a downsample whose forward ends in its K13 epilogue alone (bias, gamma^z/phi^z,
        no activation, no act quantizer), the conv's raw output and that epilogue's inputs
        instead (K.LazyRes): the block tail's fused pass applies the epilogue -- the same ops
        -- and runs its backward, two activation-sized launches fewer; anything else
        materialises it exactly as ds.forward would."""
        if (K.FOLD_RESIDUAL and K.TAIL_LAZY[0] is self and not self._forward_hooks
                and not ds._forward_hooks and ds.epilogue_fusable(x) and ds.act_code() == 0
                and not (ds.use_act_quant and not ds.disable_act_quant)):
            raw, bias = ds.forward_raw(x)
            gamma, phi = ds.affine()
            return K.LazyRes(raw, bias, gamma, phi)
        return ds(x)

    def _tail(self, last, inp, residual):
        """last(inp) (+ residual) -> block activation -> block act quant.  When `last` has
        no activation of its own and the block's is ReLU / identity, its bias add, the
        residual add and the activation run as one K13 epilogue pass (bit-identical)."""
        if (residual is not None
                and isinstance(self.activation_function, (nn.ReLU, StraightThrough))
                and isinstance(last.activation_function, StraightThrough)
                and (last.disable_act_quant or not last.use_act_quant)
                and last.epilogue_fusable(inp)):
            raw, bias = last.forward_raw(inp)
            relu = isinstance(self.activation_function, nn.ReLU)
            q = fusable_act_quantizer(self.act_quantizer, self.use_act_quant)
            gamma, phi = last.affine()
            # lazy only for the block the loop targets, and only when no hook can see the
            # placeholder output (K.TAIL_LAZY)
            lazy_ok = K.TAIL_LAZY[0] is self and not self._forward_hooks
            if gamma is not None:   # last's gamma^z/phi^z, residual, act (+ act quant)
                lazy = lazy_ok and (q is not None or not self.use_act_quant)
                out = K.epilogue(raw, bias, gamma, phi, residual, relu, q, lazy=lazy)
                if q is None and self.use_act_quant:
                    out = self.act_quantizer(out)
                return out
            if q is not None:
                # + the block's act quant in the same pass: the general epilogue with no
                # gamma^z / phi^z, whose backward sums the act delta per (n, c) row as the
                # fused tail does -- so the recon loop (BRECQ's act phase without --bias_cal)
                # takes the block's last epilogue, the loss and its backward as one pass
                # (lazy), bit-identical to this unfused form
                return K.epilogue(raw, bias, None, None, residual, relu, q, lazy=lazy_ok)
            lazy = lazy_ok and not self.use_act_quant
            out = K.bias_act(raw, bias, residual, relu, lazy=lazy)
            if self.use_act_quant:
                out = self.act_quantizer(out)
            return out
        residual = K.materialize(residual)
        out = last(inp)
        if residual is not None:
            out = out + residual
        return self._finish(out)


class QuantBasicBlock(BaseQuantBlock):
    """ResNet-18/34 block (quant_block.py:76-130)."""

    def __init__(self, basic_block, weight_quant_params: dict = {}, act_quant_params: dict = {}):
        super().__init__(act_quant_params)
        self.conv1 = QuantModule(basic_block.conv1, weight_quant_params, act_quant_params)
        self.conv1.activation_function = basic_block.relu1
        self.conv2 = QuantModule(basic_block.conv2, weight_quant_params, act_quant_params,
                                 disable_act_quant=True)
        self.activation_function = basic_block.relu2
        self.downsample = None if basic_block.downsample is None else QuantModule(
            basic_block.downsample[0], weight_quant_params, act_quant_params, disable_act_quant=True)
        self.stride = basic_block.stride

    def forward(self, x):
        if self.cache_features == 'if':
            self.cached_inp_features += [self._cache(x)]
        residual = x if self.downsample is None else self._residual(self.downsample, x)
        # conv1's output feeds conv2 only: its epilogue may fold into conv2's im2col GEMM
        # (kernels.EPI_CONSUMER; conv2 materialises it when it does not run as that GEMM)
        fold = (K.EPI_INTO_GEMM and torch.is_grad_enabled() and x.is_cuda
                and not self._forward_hooks and not self._forward_pre_hooks
                and not self.conv2._forward_pre_hooks and self.conv2.cache_features == 'none')
        prev = K.EPI_CONSUMER[0]
        K.EPI_CONSUMER[0] = self.conv2 if fold else None
        try:
            out1 = self.conv1(x)
        finally:
            K.EPI_CONSUMER[0] = prev
        out = self._tail(self.conv2, out1, residual)
        if self.cache_features == 'of':
            self.cached_out_features += [self._cache(out)]
        return out

    def input_readers(self):
        return None if self.downsample is None else [self.conv1, self.downsample]

    def identity_input_convs(self):
        return [self.conv1] if self.downsample is None else None

    def toggleHardTarget(self):
        for m in (self.conv1, self.conv2, self.downsample):
            if m is not None:
                m.weight_quantizer.hard_targets = not m.weight_quantizer.hard_targets


class QuantBottleneck(BaseQuantBlock):
    """ResNet-50 block (quant_block.py:133-166)."""

    def __init__(self, bottleneck, weight_quant_params: dict = {}, act_quant_params: dict = {}):
        super().__init__(act_quant_params)
        self.conv1 = QuantModule(bottleneck.conv1, weight_quant_params, act_quant_params)
        self.conv1.activation_function = bottleneck.relu1
        self.conv2 = QuantModule(bottleneck.conv2, weight_quant_params, act_quant_params)
        self.conv2.activation_function = bottleneck.relu2
        self.conv3 = QuantModule(bottleneck.conv3, weight_quant_params, act_quant_params,
                                 disable_act_quant=True)
        self.activation_function = bottleneck.relu3
        self.downsample = None if bottleneck.downsample is None else QuantModule(
            bottleneck.downsample[0], weight_quant_params, act_quant_params, disable_act_quant=True)
        self.stride = bottleneck.stride

    def input_readers(self):
        return None if self.downsample is None else [self.conv1, self.downsample]

    def identity_input_convs(self):
        return [self.conv1] if self.downsample is None else None

    def forward(self, x):
        if self.cache_features == 'if':
            self.cached_inp_features += [self._cache(x)]
        residual = x if self.downsample is None else self._residual(self.downsample, x)
        out = self._tail(self.conv3, self.conv2(self.conv1(x)), residual)
        if self.cache_features == 'of':
            self.cached_out_features += [self._cache(out)]
        return out


class QuantResBottleneckBlock(BaseQuantBlock):
    """RegNetX block without SE (quant_block.py:169-202): f.a / f.b / f.c + optional proj."""

    def __init__(self, bottleneck, weight_quant_params: dict = {}, act_quant_params: dict = {}):
        super().__init__(act_quant_params)
        self.conv1 = QuantModule(bottleneck.f.a, weight_quant_params, act_quant_params)
        self.conv1.activation_function = bottleneck.f.a_relu
        self.conv2 = QuantModule(bottleneck.f.b, weight_quant_params, act_quant_params)
        self.conv2.activation_function = bottleneck.f.b_relu
        self.conv3 = QuantModule(bottleneck.f.c, weight_quant_params, act_quant_params,
                                 disable_act_quant=True)
        self.activation_function = bottleneck.relu
        self.downsample = QuantModule(bottleneck.proj, weight_quant_params, act_quant_params,
                                      disable_act_quant=True) if bottleneck.proj_block else None
        self.proj_block = bottleneck.proj_block

    def input_readers(self):
        return [self.conv1, self.downsample] if self.proj_block else None

    def identity_input_convs(self):
        return None if self.proj_block else [self.conv1]

    def forward(self, x):
        if self.cache_features == 'if':
            self.cached_inp_features += [self._cache(x)]
        residual = self._residual(self.downsample, x) if self.proj_block else x
        out = self._tail(self.conv3, self.conv2(self.conv1(x)), residual)
        if self.cache_features == 'of':
            self.cached_out_features += [self._cache(out)]
        return out


class QuantInvertedResidual(BaseQuantBlock):
    """MobileNetV2 block (quant_block.py:205-239); no activation after the residual add."""

    def __init__(self, inv_res, weight_quant_params: dict = {}, act_quant_params: dict = {}):
        super().__init__(act_quant_params)
        self.use_res_connect = inv_res.use_res_connect
        self.expand_ratio = inv_res.expand_ratio
        if self.expand_ratio == 1:
            self.conv = nn.Sequential(
                QuantModule(inv_res.conv[0], weight_quant_params, act_quant_params),
                QuantModule(inv_res.conv[3], weight_quant_params, act_quant_params,
                            disable_act_quant=True))
            self.conv[0].activation_function = nn.ReLU6()
        else:
            self.conv = nn.Sequential(
                QuantModule(inv_res.conv[0], weight_quant_params, act_quant_params),
                QuantModule(inv_res.conv[3], weight_quant_params, act_quant_params),
                QuantModule(inv_res.conv[6], weight_quant_params, act_quant_params,
                            disable_act_quant=True))
            self.conv[0].activation_function = nn.ReLU6()
            self.conv[1].activation_function = nn.ReLU6()

    def input_readers(self):
        return None if self.use_res_connect else [self.conv[0]]

    def identity_input_convs(self):
        return [self.conv[0]] if self.use_res_connect else None

    def forward(self, x):
        if self.cache_features == 'if':
            self.cached_inp_features += [self._cache(x)]
        h = x
        for m in list(self.conv)[:-1]:
            h = m(h)
        # x + conv(x): fp32 addition commutes, so the fused (conv + bias) + x is bit-identical
        out = self._tail(self.conv[-1], h, x if self.use_res_connect else None)
        if self.cache_features == 'of':
            self.cached_out_features += [self._cache(out)]
        return out


specials = {
    nets.BasicBlock: QuantBasicBlock,
    nets.Bottleneck: QuantBottleneck,
    nets.InvertedResidual: QuantInvertedResidual,
    nets.ResBottleneckBlock: QuantResBottleneckBlock,
}


def register_block(fp_block_type, quant_block_type):
    """Map another FP block class (e.g. a model zoo's own BasicBlock) to a quant block."""
    specials[fp_block_type] = quant_block_type
