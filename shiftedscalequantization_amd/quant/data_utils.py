"""Block/layer feature capture for reconstruction (reference: quant/data_utils.py).

Hooked forwards capture the block input (quantized network up to the block when asym)
and its FP output.  The reference copies every batch to the host and back
(data_utils.py:29,35); here batches stay in HBM (288 GB per MI355X) and are concatenated
once -- the same values without the PCIe round trip.
"""
from typing import Union

import torch
import torch.nn.functional as F

from .quant_block import BaseQuantBlock
from .quant_layer import QuantModule
from .quant_model import QuantModel


def save_inp_oup_data(model: QuantModel, layer: Union[QuantModule, BaseQuantBlock],
                      cali_data: torch.Tensor, asym: bool = False, act_quant: bool = False,
                      batch_size: int = 32, keep_gpu: bool = True):
    device = next(model.parameters()).device
    get_inp_out = GetLayerInpOut(model, layer, device=device, asym=asym, act_quant=act_quant)
    inps, outs = [], []
    for i in range(int(cali_data.size(0) / batch_size)):
        cur_inp, cur_out = get_inp_out(cali_data[i * batch_size:(i + 1) * batch_size])
        inps.append(cur_inp)
        outs.append(cur_out)
    cached_inps, cached_outs = torch.cat(inps), torch.cat(outs)
    if not keep_gpu:
        cached_inps, cached_outs = cached_inps.cpu(), cached_outs.cpu()
    return cached_inps, cached_outs


def save_grad_data(model: QuantModel, layer: Union[QuantModule, BaseQuantBlock],
                   cali_data: torch.Tensor, damping: float = 1., act_quant: bool = False,
                   batch_size: int = 32, keep_gpu: bool = True):
    """data_utils.py:40-71 (Fisher capture; only used by opt_mode != 'mse')."""
    device = next(model.parameters()).device
    get_grad = GetLayerGrad(model, layer, device, act_quant=act_quant)
    grads = [get_grad(cali_data[i * batch_size:(i + 1) * batch_size])
             for i in range(int(cali_data.size(0) / batch_size))]
    cached_grads = torch.cat(grads).abs() + 1.0
    return cached_grads if keep_gpu else cached_grads.cpu()


class StopForwardException(Exception):
    pass


class DataSaverHook:
    def __init__(self, store_input=False, store_output=False, stop_forward=False):
        self.store_input = store_input
        self.store_output = store_output
        self.stop_forward = stop_forward
        self.input_store = None
        self.output_store = None

    def __call__(self, module, input_batch, output_batch):
        if self.store_input:
            self.input_store = input_batch
        if self.store_output:
            self.output_store = output_batch
        if self.stop_forward:
            raise StopForwardException


class GetLayerInpOut:
    def __init__(self, model: QuantModel, layer, device: torch.device, asym: bool = False,
                 act_quant: bool = False):
        self.model = model
        self.layer = layer
        self.asym = asym
        self.device = device
        self.act_quant = act_quant
        self.data_saver = DataSaverHook(store_input=True, store_output=True, stop_forward=True)

    def __call__(self, model_input):
        self.model.eval()
        self.model.set_quant_state(False, False)
        handle = self.layer.register_forward_hook(self.data_saver)
        with torch.no_grad():
            try:
                _ = self.model(model_input.to(self.device))
            except StopForwardException:
                pass
            if self.asym:
                self.data_saver.store_output = False
                self.model.set_quant_state(weight_quant=True, act_quant=self.act_quant)
                try:
                    _ = self.model(model_input.to(self.device))
                except StopForwardException:
                    pass
                self.data_saver.store_output = True
        handle.remove()
        self.model.set_quant_state(False, False)
        self.layer.set_quant_state(True, self.act_quant)
        self.model.train()
        return self.data_saver.input_store[0].detach(), self.data_saver.output_store.detach()


class GradSaverHook:
    def __init__(self, store_grad=True):
        self.store_grad = store_grad
        self.stop_backward = False
        self.grad_out = None

    def __call__(self, module, grad_input, grad_output):
        if self.store_grad:
            self.grad_out = grad_output[0]
        if self.stop_backward:
            raise StopForwardException


class GetLayerGrad:
    def __init__(self, model: QuantModel, layer, device: torch.device, act_quant: bool = False):
        self.model = model
        self.layer = layer
        self.device = device
        self.act_quant = act_quant
        self.data_saver = GradSaverHook(True)

    def __call__(self, model_input):
        self.model.eval()
        handle = self.layer.register_full_backward_hook(self.data_saver)
        with torch.enable_grad():
            try:
                self.model.zero_grad()
                inputs = model_input.to(self.device)
                self.model.set_quant_state(False, False)
                out_fp = self.model(inputs)
                quantize_model_till(self.model, self.layer, self.act_quant)
                out_q = self.model(inputs)
                loss = F.kl_div(F.log_softmax(out_q, dim=1), F.softmax(out_fp, dim=1),
                                reduction='batchmean')
                loss.backward()
            except StopForwardException:
                pass
        handle.remove()
        self.model.set_quant_state(False, False)
        self.layer.set_quant_state(True, self.act_quant)
        self.model.train()
        return self.data_saver.grad_out.data


def quantize_model_till(model, layer, act_quant: bool = False):
    model.set_quant_state(False, False)
    for name, module in model.named_modules():
        if isinstance(module, (QuantModule, BaseQuantBlock)):
            module.set_quant_state(True, act_quant)
        if module == layer:
            break
