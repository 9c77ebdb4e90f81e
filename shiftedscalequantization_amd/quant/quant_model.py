"""QuantModel (reference: quant/quant_model.py): fold BN, then recursively replace
Conv2d/Linear by QuantModule and known residual blocks by quant blocks."""
import torch
import torch.nn as nn

from .. import kernels as K
from .fold_bn import search_fold_and_remove_bn
from .quant_block import BaseQuantBlock, specials
from .quant_layer import QuantModule, StraightThrough


class QuantModel(nn.Module):
    def __init__(self, model: nn.Module, weight_quant_params: dict = {}, act_quant_params: dict = {}):
        super().__init__()
        search_fold_and_remove_bn(model)
        self.model = model
        self.quant_module_refactor(self.model, weight_quant_params, act_quant_params)
        self.qState = []

    def quant_module_refactor(self, module: nn.Module, weight_quant_params: dict = {},
                              act_quant_params: dict = {}, depth=0, moduleName=''):
        """quant_model.py:15-44."""
        prev_quantmodule = None
        for name, child_module in module.named_children():
            curName = moduleName + '.' + name
            if name in ['relu2']:
                continue
            if type(child_module) in specials:
                setattr(module, name, specials[type(child_module)](child_module, weight_quant_params,
                                                                   act_quant_params))
                getattr(module, name).setPathName(curName)
            elif isinstance(child_module, (nn.Conv2d, nn.Linear)):
                setattr(module, name, QuantModule(child_module, weight_quant_params, act_quant_params))
                prev_quantmodule = getattr(module, name)
                prev_quantmodule.pathName = curName
            elif isinstance(child_module, (nn.ReLU, nn.ReLU6)):
                if prev_quantmodule is not None:
                    prev_quantmodule.activation_function = child_module
                    setattr(module, name, StraightThrough())
            elif isinstance(child_module, StraightThrough):
                continue
            elif type(child_module) is nn.MaxPool2d and K.MAXPOOL_HIP:
                # the stem's pool on ssq_maxpool2d_fwd (same results as torch's)
                setattr(module, name, K.SsqMaxPool2d.wrap(child_module))
            else:
                self.quant_module_refactor(child_module, weight_quant_params, act_quant_params,
                                           depth + 1, moduleName=curName)

    def set_quant_state(self, weight_quant: bool = False, act_quant: bool = False):
        for m in self.model.modules():
            if isinstance(m, (QuantModule, BaseQuantBlock)):
                m.set_quant_state(weight_quant, act_quant)

    def set_quant_init_state(self):
        for m in self.model.modules():
            if isinstance(m, (QuantModule, BaseQuantBlock)):
                m.set_quant_init_state()

    def forward(self, input):
        return self.model(input)

    def _quant_modules(self):
        return [m for m in self.model.modules() if isinstance(m, QuantModule)]

    def set_first_last_layer_to_8bit(self):
        """quant_model.py:59-69."""
        ms = self._quant_modules()
        ms[0].weight_quantizer.bitwidth_refactor(8)
        ms[0].act_quantizer.bitwidth_refactor(8)
        ms[-1].weight_quantizer.bitwidth_refactor(8)
        ms[-2].act_quantizer.bitwidth_refactor(8)
        ms[0].ignore_reconstruction = True

    def disable_network_output_quantization(self):
        self._quant_modules()[-1].disable_act_quant = True

    def disable_cache_features(self):
        for m in self.model.modules():
            if isinstance(m, (QuantModule, BaseQuantBlock)):
                m.disable_cache_features()

    def clear_cached_features(self):
        for m in self.model.modules():
            if isinstance(m, (QuantModule, BaseQuantBlock)):
                m.clear_cached_features()

    def store_quantization_state(self):
        self.qState = [m.use_weight_quant for m in self.modules() if isinstance(m, QuantModule)]

    def restore_quantization_state(self):
        for m, s in zip([m for m in self.modules() if isinstance(m, QuantModule)], self.qState):
            m.use_weight_quant = s

    def synchorize_activation_statistics(self):
        """All-average of the activation deltas across ranks after the act init forward --
        the reference's intent (quant_model.py:78-83, linklink call commented out; called
        by Brecq/main_imagenet_dist.py:210-211).  Two additions keep the act quantizers
        replicated, which the loop's gradient all-reduce assumes: the blocks' own output
        quantizers (BaseQuantBlock.act_quantizer) are averaged too, and the zero points --
        integers from each rank's own shard, 0 after a ReLU -- are taken from rank 0."""
        from ..parallel_dp import all_average_, broadcast_
        from .quant_block import BaseQuantBlock
        for m in self.modules():
            if isinstance(m, (QuantModule, BaseQuantBlock)):
                aq = m.act_quantizer
                if getattr(aq, 'delta', None) is not None and getattr(aq, 'inited', True):
                    all_average_(aq.delta.data)
                    if getattr(aq, 'zero_point', None) is not None and torch.is_tensor(aq.zero_point):
                        broadcast_(aq.zero_point.data, 0)
