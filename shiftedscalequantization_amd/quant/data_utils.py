"""Device-resident feature and gradient capture for the BRECQ loops (reference:
quant/data_utils.py:8-71, the SURVEY §8(f) row-1 feature cache).

What is captured is the reference's: for a module (layer or block) over the calibration
set, its full-precision output and its input -- with `asym`, the input as the network
quantized up to the module produces it (weights, plus activations with `act_quant`); and
for the Fisher losses the gradient of the KL(quantized-up-to-module || FP) loss at the
module's output, stored as |g| + 1.

How differs: the reference keeps one hook object per call, copies every batch to the host
and back, and concatenates.  Here a forward hook writes each batch straight into a buffer
allocated once on the device for the whole calibration set (288 GB of HBM per MI355X; the
largest ResNet cache is 822 MB), then stops the forward -- nothing after the module runs.
With data parallelism each rank calls this on its own shard of the samples.
"""
from typing import Union

import torch
import torch.nn.functional as F

from .quant_block import BaseQuantBlock
from .quant_layer import QuantModule
from .quant_model import QuantModel


class StopForwardException(Exception):
    """Raised by a capture hook once its module has run (the rest of the forward is not
    needed).  Also raised by drivers.cache_block_features' stop hook."""


class _RowSink:
    """Rows [at, at + batch) of a (n_rows, ...) device buffer created on first write."""

    def __init__(self, n_rows):
        self.n_rows = n_rows
        self.buf = None
        self.at = 0

    def write(self, t):
        t = t.detach()
        if self.buf is None:
            self.buf = torch.empty((self.n_rows,) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
        self.buf[self.at:self.at + t.shape[0]].copy_(t)


class _CaptureHook:
    """Forward hook: module input into `inp`, output into `out` (either may be None), then
    stop the forward."""

    def __init__(self, inp=None, out=None):
        self.inp, self.out = inp, out

    def __call__(self, module, args, output):
        if self.inp is not None:
            self.inp.write(args[0])
        if self.out is not None:
            self.out.write(output)
        raise StopForwardException


def _forward_until(model, module, batch, hook):
    handle = module.register_forward_hook(hook)
    try:
        with torch.no_grad():
            model(batch)
    except StopForwardException:
        pass
    finally:
        handle.remove()


def save_inp_oup_data(model: QuantModel, layer: Union[QuantModule, BaseQuantBlock],
                      cali_data: torch.Tensor, asym: bool = False, act_quant: bool = False,
                      batch_size: int = 32, keep_gpu: bool = True):
    """data_utils.py:8-37 -> (cached inputs, cached FP outputs) of `layer`, whole batches
    of `cali_data` only (as the reference's int(N / batch_size) loop)."""
    device = next(model.parameters()).device
    nb = int(cali_data.size(0) / batch_size)
    out = _RowSink(nb * batch_size)
    inp = _RowSink(nb * batch_size)
    fp_hook = _CaptureHook(inp=None if asym else inp, out=out)
    q_hook = _CaptureHook(inp=inp) if asym else None
    model.eval()
    for i in range(nb):
        batch = cali_data[i * batch_size:(i + 1) * batch_size].to(device)
        out.at = inp.at = i * batch_size
        model.set_quant_state(False, False)
        _forward_until(model, layer, batch, fp_hook)
        if asym:
            model.set_quant_state(weight_quant=True, act_quant=act_quant)
            _forward_until(model, layer, batch, q_hook)
    model.set_quant_state(False, False)
    layer.set_quant_state(True, act_quant)
    model.train()
    if nb == 0:
        return None, None
    if keep_gpu:
        return inp.buf, out.buf
    return inp.buf.cpu(), out.buf.cpu()


def quantize_model_till(model, layer, act_quant: bool = False):
    """Quantize every module up to and including `layer` (modules are in forward order
    for every model here), nothing after it."""
    model.set_quant_state(False, False)
    for module in model.modules():
        if isinstance(module, (QuantModule, BaseQuantBlock)):
            module.set_quant_state(True, act_quant)
        if module is layer:
            break


def save_grad_data(model: QuantModel, layer: Union[QuantModule, BaseQuantBlock],
                   cali_data: torch.Tensor, damping: float = 1., act_quant: bool = False,
                   batch_size: int = 32, keep_gpu: bool = True):
    """data_utils.py:40-71 (Fisher losses only): per batch, the gradient at `layer`'s
    output of KL(log_softmax(quantized-till-layer output) || softmax(FP output)),
    'batchmean'; returned as |g| + 1 for the whole calibration set."""
    device = next(model.parameters()).device
    nb = int(cali_data.size(0) / batch_size)
    sink = _RowSink(nb * batch_size)

    def grad_hook(module, grad_input, grad_output):
        sink.write(grad_output[0])

    model.eval()
    handle = layer.register_full_backward_hook(grad_hook)
    try:
        for i in range(nb):
            sink.at = i * batch_size
            x = cali_data[i * batch_size:(i + 1) * batch_size].to(device)
            with torch.enable_grad():
                model.zero_grad()
                model.set_quant_state(False, False)
                out_fp = model(x)
                quantize_model_till(model, layer, act_quant)
                out_q = model(x)
                F.kl_div(F.log_softmax(out_q, dim=1), F.softmax(out_fp, dim=1),
                         reduction='batchmean').backward()
    finally:
        handle.remove()
    model.set_quant_state(False, False)
    layer.set_quant_state(True, act_quant)
    model.train()
    if nb == 0:
        return None
    grads = sink.buf.abs() + 1.0
    return grads if keep_gpu else grads.cpu()
