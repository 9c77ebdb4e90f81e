"""Host orchestration of a calibration run (reference: myScaledMethods.py:17-120,263-307,
ShiftedScaleQuant.py:12-59,119-286, Brecq/main_imagenet.py:204-244).

Same helper names as the reference.  Feature caching forwards stop at the block being
cached (a forward hook raises, as in quant/data_utils.py) instead of running the whole
network twice per block, and cached tensors stay in HBM.
"""
import torch
import torch.nn as nn

from . import nets
from .quant import (BaseQuantBlock, ChannelQuant, ChannelQuantMSE, QuantModel, QuantModule,
                    UniformAffineQuantizer, block_recon_fused_shiftedScale, block_reconstruction,
                    layer_recon_fused_shiftedScale, layer_reconstruction)
from .quant.data_utils import StopForwardException


# ------------------------------------------------------------------ builders (myScaledMethods.py)
def build_ShiftedChannelQuantMSELayer(model, curName, layer, delta=1.0, **kwargs):
    layer.weight_quantizer = ChannelQuantMSE(delta, uaq=layer.weight_quantizer,
                                             weight_tensor=layer.org_weight.data,
                                             shiftTarget=kwargs['shiftTarget'], opt_mode=kwargs['opt_mode'],
                                             level=kwargs['level'], threshold=kwargs['threshold'],
                                             name=curName)
    layer.use_weight_quant = True
    layer.cache_features = 'none'
    layer.weight_quantizer.init_scale(layer.org_weight.data)


def build_ShiftedChannelQuantMSEBlock(model, prv_name, block, delta=1.0, **kwargs):
    """myScaledMethods.py:27-40: every direct QuantModule child still on a UAQ."""
    for name, layer in block.named_children():
        if isinstance(layer, QuantModule) and isinstance(layer.weight_quantizer, UniformAffineQuantizer):
            build_ShiftedChannelQuantMSELayer(model, prv_name + '.' + name, layer, delta, **kwargs)


def build_ShiftedChannelQuantMSE(model, layerDisabled, prv_name="", delta=1.0, **kwargs):
    """The nested builder of channelShift_wMSE (ShiftedScaleQuant.py:155-173), walk as
    written: a QuantModule gets a ChannelQuantMSE unless it is ignore_reconstruction or
    listed in layerDisabled; a QuantBasicBlock listed in layerDisabled has ALL its layers
    built (the reference's inverted test, kept), otherwise it is recursed into."""
    from .quant.quant_block import QuantBasicBlock
    for name, module in model.named_children():
        curName = prv_name + '.' + name
        if isinstance(module, QuantModule):
            if module.ignore_reconstruction:
                continue
            if curName not in layerDisabled:
                build_ShiftedChannelQuantMSELayer(model, curName, module, delta, **kwargs)
        elif isinstance(module, QuantBasicBlock):
            if module.ignore_reconstruction:
                continue
            if curName in layerDisabled:
                build_ShiftedChannelQuantMSEBlock(model, curName, module, delta, **kwargs)
            else:
                build_ShiftedChannelQuantMSE(module, layerDisabled, curName, delta, **kwargs)
        else:
            build_ShiftedChannelQuantMSE(module, layerDisabled, curName, delta, **kwargs)


def channelShift_wMSE(qnn, cali_data, level=1, threshold=1.0, opt_mode='max',
                      shiftTarget=(31 / 32, 33 / 32, 1.0), layerDisabled=('.model.fc',),
                      init_samples=64):
    """ShiftedScaleQuant.py:119-183, the path the shipped entry point runs (`--test=True`,
    :361): weight-quant init on cali[:64], then per-(Ci,kh,kw) input scales chosen by
    ChannelQuantMSE.init_scale (K10) for every reconstructable layer but the fc.  No
    reconstruction loop; returns the quantized model (weight quant on, act quant off)."""
    qnn.set_quant_state(True, False)
    with torch.no_grad():
        qnn(cali_data[:init_samples])
    build_ShiftedChannelQuantMSE(qnn, list(layerDisabled), '', delta=1.0, shiftTarget=list(shiftTarget),
                                 level=level, threshold=threshold, opt_mode=opt_mode)
    return qnn


def build_ShiftedChannelQuantLayer(model, curName, layer, delta=1.0, **kwargs):
    skip = tuple(kwargs.get('skipShiftLayer', []))
    shiftTarget = kwargs['shiftTarget'] if not (skip and curName.startswith(skip)) else [2 / 2]
    layer.weight_quantizer = ChannelQuant(delta, uaq=layer.weight_quantizer,
                                          weight_tensor=layer.org_weight.data,
                                          shiftTarget=shiftTarget, name=curName)
    layer.use_weight_quant = True
    layer.cache_features = 'none'


def build_ShiftedChannelQuantBlock(model, prv_name, block, delta=1.0, **kwargs):
    for name, layer in block.named_modules():
        if name and isinstance(layer, QuantModule) and isinstance(layer.weight_quantizer,
                                                                  UniformAffineQuantizer):
            build_ShiftedChannelQuantLayer(model, prv_name + '.' + name, layer, delta, **kwargs)


def build_ShiftedChannelQuant(model: nn.Module, layerEnabled, prv_name="", delta=1.0, **kwargs):
    """myScaledMethods.py:59-75 (any BaseQuantBlock, not only QuantBasicBlock)."""
    for name, module in model.named_children():
        curName = prv_name + '.' + name
        if isinstance(module, QuantModule):
            if module.ignore_reconstruction:
                continue
            if curName in layerEnabled:
                build_ShiftedChannelQuantLayer(model, curName, module, delta, **kwargs)
        elif isinstance(module, BaseQuantBlock):
            if module.ignore_reconstruction:
                continue
            if curName in layerEnabled:
                build_ShiftedChannelQuantBlock(model, curName, module, delta, **kwargs)
            else:
                build_ShiftedChannelQuant(module, layerEnabled, curName, delta, **kwargs)
        else:
            build_ShiftedChannelQuant(module, layerEnabled, curName, delta, **kwargs)


def set_quant_state_block(model, layers, prv_name='', state=False, act=False):
    """myScaledMethods.py:91-108."""
    for name, module in model.named_children():
        curName = prv_name + '.' + name
        if isinstance(module, QuantModule):
            if module.ignore_reconstruction:
                continue
            if curName in layers:
                if act:
                    module.use_act_quant = state
                else:
                    module.use_weight_quant = state
        elif isinstance(module, BaseQuantBlock):
            if module.ignore_reconstruction:
                continue
            if curName in layers:
                module.set_quant_state_block(state, act)
        else:
            set_quant_state_block(module, layers, curName, state, act)


def set_cache_state(model, layers, prv_name='', state='none'):
    """myScaledMethods.py:110-120."""
    for name, module in model.named_children():
        curName = prv_name + '.' + name
        if curName in layers:
            if module.ignore_reconstruction:
                continue
            module.cache_features = state
        elif isinstance(module, QuantModule):
            continue
        else:
            set_cache_state(module, layers, curName, state)


def find_module(model, path):
    for name, m in model.named_modules():
        if '.' + name == path or name == path.lstrip('.'):
            return m
    raise KeyError(path)


def _stop_after(module):
    def hook(m, i, o):
        raise StopForwardException
    return module.register_forward_hook(hook)


@torch.no_grad()
def cache_block_features(qnn, path, cali_data, batch_size, device):
    """ShiftedScaleQuant.py:243-255: cache the block's input with the current quant state and
    its FP output; each forward stops right after the block."""
    module = find_module(qnn, path)
    h = _stop_after(module)
    try:
        set_cache_state(qnn, [path], prv_name='', state='if')
        for i in range(len(cali_data) // batch_size):
            try:
                qnn(cali_data[i * batch_size:(i + 1) * batch_size].to(device))
            except StopForwardException:
                pass
        qnn.store_quantization_state()
        qnn.set_quant_state(False, False)
        set_cache_state(qnn, [path], prv_name='', state='of')
        for i in range(len(cali_data) // batch_size):
            try:
                qnn(cali_data[i * batch_size:(i + 1) * batch_size].to(device))
            except StopForwardException:
                pass
        qnn.restore_quantization_state()
        set_cache_state(qnn, [path], prv_name='', state='none')
    finally:
        h.remove()
    return module


def run_ShiftReconFused(model, curName, module, qnn, test_loader, act=False, **kwargs):
    """ShiftedScaleQuant.py:48-59."""
    lmda = (kwargs.get('lmdaR', 0.01), kwargs['lmda'])
    common = dict(act=act, bias_cal=kwargs.get('bias_cal', False), verbose=kwargs.get('verbose', True))
    if isinstance(module, QuantModule):
        return [layer_recon_fused_shiftedScale(module, kwargs['iters'], lmda, qnn, test_loader, **common)]
    if isinstance(module, BaseQuantBlock):
        return [block_recon_fused_shiftedScale(module, kwargs['iters'], lmda, qnn, test_loader, **common)]
    raise ValueError('Not supported reconstruction module type: {}'.format(type(module)))


def QuantRecursiveShiftRecon(model, layerEnabled, qnn, test_loader, prv_name="", ret=None, act=False,
                             **kwargs):
    """ShiftedScaleQuant.py:12-29."""
    ret = {} if ret is None else ret
    for name, module in model.named_children():
        curName = prv_name + '.' + name
        if isinstance(module, (QuantModule, BaseQuantBlock)):
            if module.ignore_reconstruction:
                continue
            if curName in layerEnabled:
                ret[curName] = run_ShiftReconFused(model, curName, module, qnn, test_loader, act, **kwargs)
            elif isinstance(module, BaseQuantBlock):
                QuantRecursiveShiftRecon(module, layerEnabled, qnn, test_loader, curName, ret, act, **kwargs)
        else:
            QuantRecursiveShiftRecon(module, layerEnabled, qnn, test_loader, curName, ret, act, **kwargs)
    return ret


def block_paths(qnn):
    """Paths ('.model.layer1.0', ...) of every reconstructable block, in forward order."""
    return ['.' + n for n, m in qnn.named_modules()
            if isinstance(m, BaseQuantBlock) and not m.ignore_reconstruction]


def build_qnn(arch, n_bits_w, n_bits_a, channel_wise=True, w_scale_method='mse',
              a_scale_method='mse', device='cuda', checkpoint='', disable_8bit_head_stem=False):
    """myScaledMethods.py:263-307 (random-init weights unless a checkpoint is given)."""
    cnn = nets.ARCHS[arch]()
    if checkpoint:
        cnn.load_state_dict(torch.load(checkpoint, map_location='cpu', weights_only=True))
    cnn.to(device).eval()
    wq = {'n_bits': n_bits_w, 'channel_wise': channel_wise, 'scale_method': w_scale_method,
          'tune_delta_zero': False, 'symmetric': False}
    aq = {'n_bits': n_bits_a, 'channel_wise': False, 'scale_method': a_scale_method,
          'tune_delta_zero': False, 'leaf_param': True, 'symmetric': False}
    qnn = QuantModel(model=cnn, weight_quant_params=wq, act_quant_params=aq).to(device).eval()
    if not disable_8bit_head_stem:
        qnn.set_first_last_layer_to_8bit()
    return qnn


def recon_model(qnn, model, **kwargs):
    """Brecq/main_imagenet.py:204-224: BRECQ block/layer reconstruction over the model."""
    for name, module in model.named_children():
        if isinstance(module, QuantModule):
            if module.ignore_reconstruction:
                continue
            layer_reconstruction(qnn, module, **kwargs)
        elif isinstance(module, BaseQuantBlock):
            if module.ignore_reconstruction:
                continue
            block_reconstruction(qnn, module, **kwargs)
        else:
            recon_model(qnn, module, **kwargs)
