"""Packed low-bit export of a calibrated QuantModel.

The reference persists a calibrated network as an fp32 `state_dict` (main_cifar10.py:86)
plus the pickled per-layer shift choice (myScaledMethods.py:204-205, restored by
ShiftedScaleQuant.py:31-45).  Here every reconstructed weight is stored as its integer
codes, packed 2/4/8 bits per code (ssq_pack_encode, K15), with the per-channel vectors its
quantizer dequantizes with:

    W_hat = ((q - zero_point[co]) * scale[co | co,ci]) (* col_scale[j])

plus conv bias, gamma^z/phi^z and the activation quantizer's (delta, zero_point).  The
encoder verifies on the device that decoding reproduces the quantizer's own hard output
bit for bit; a quantizer that is still soft (recon not finalised) is refused.
`load_quantized` decodes with ssq_pack_decode (K16) and installs each weight as a
`PackedWeight` quantizer, so the restored model's forward equals the calibrated one's.
"""
import json

import torch
import torch.nn as nn

from .. import kernels as K
from .adaptive_rounding import AdaRoundQuantizer
from .channelQuant import ChannelQuant
from .channelQuantMSE import ChannelQuantMSE
from .quant_layer import QuantModule, UniformAffineQuantizer

FORMAT = "ssq-packed-v1"


def _per_co(t, Co):
    t = t.detach().reshape(-1).float()
    return t.expand(Co).contiguous() if t.numel() == 1 else t.contiguous()


def _scaled(delta, scale, Co, Ci):
    """fp32(delta * scale) flattened, and whether it is per (co, ci)."""
    d = delta.detach().float()
    if float(scale) != 1.0:
        d = d * float(scale)
    per_ci = d.numel() == Co * Ci and d.numel() != Co
    return (d.reshape(-1).contiguous() if per_ci else _per_co(d, Co)), per_ci


@torch.no_grad()
def dequant_form(module: QuantModule):
    """(W_hat, fields) of a QuantModule's hard weight quantizer: W_hat is what the
    module's forward uses, fields the (zero_point, scale, per_ci, col_scale, n_bits, qmin,
    qmax, kind) it dequantizes with."""
    q = module.weight_quantizer
    w = module.weight.detach()
    Co, Ci = int(w.shape[0]), int(w.shape[1])
    col = None
    if type(q) is UniformAffineQuantizer:
        what = q(w)
        qmin, qmax = K.qrange(q.n_bits, q.sym)
        zp, (d1, per_ci) = _per_co(q.zero_point, Co), _scaled(q.delta, 1.0, Co, Ci)
        kind = "uaq"
    elif isinstance(q, ChannelQuant):
        soft = {"adaShift": not (q.hard_targets and q.hard_round),
                "learned_hard_sigmoid": not q.hard_targets,
                "adaround": not q.hard_round}.get(q.opt_mode, False)
        if soft:
            raise ValueError(f"{module.pathName or 'layer'}: ChannelQuant is still soft "
                             f"(mode {q.opt_mode}); finish the reconstruction first")
        what = q(w)
        qmin, qmax = K.qrange(q.n_bits, q.sym)
        zp = _per_co(q.zero_point, Co)
        if q.opt_mode == "adaShift":
            d1, per_ci = _per_co(q._src_delta, Co), False
        elif q.opt_mode in "learned_hard_sigmoid":
            d1, per_ci = q.get_delta().reshape(-1).contiguous(), True
        else:   # 'adaround' / 'none'
            d1, per_ci = _scaled(q.delta, q.shiftedScale, Co, Ci)
        kind = f"channelquant:{q.opt_mode}"
    elif isinstance(q, AdaRoundQuantizer):
        if q.round_mode == "learned_hard_sigmoid" and q.soft_targets:
            raise ValueError(f"{module.pathName or 'layer'}: AdaRoundQuantizer still has soft "
                             "targets; finish the reconstruction first")
        what = q(w)
        qmin, qmax = 0, 2 ** q.n_bits - 1
        zp, (d1, per_ci) = _per_co(q.zero_point, Co), _scaled(q.delta, 1.0, Co, Ci)
        kind = f"adaround:{q.round_mode}"
    elif isinstance(q, ChannelQuantMSE):
        what = q(w)
        qmin, qmax = 0, 2 ** q.n_bits - 1
        d1, per_ci = _per_co(q.delta, Co), False
        zp = torch.round(_per_co(q.raw_zero_point, Co) / d1)
        col = q.inp_scale.detach().reshape(-1).float().contiguous()
        kind = "channelquantmse"
    elif isinstance(q, PackedWeight):
        return q(w), q.fields()
    else:
        raise TypeError(f"no packed export for weight quantizer {type(q).__name__}")
    return what, dict(zero_point=zp, scale=d1, per_ci=per_ci, col_scale=col, n_bits=q.n_bits,
                      qmin=qmin, qmax=qmax, kind=kind)


class PackedWeight(nn.Module):
    """Weight 'quantizer' of a restored model: the packed codes decoded once (K16)."""

    def __init__(self, packed, shape, zero_point, scale, per_ci, col_scale, n_bits, qmin, qmax,
                 kind):
        super().__init__()
        self.register_buffer("packed", packed)
        self.register_buffer("zero_point", zero_point)
        self.register_buffer("scale", scale)
        self.register_buffer("col_scale", col_scale)
        self.shape, self.per_ci, self.n_bits = tuple(shape), bool(per_ci), int(n_bits)
        self.qmin, self.qmax, self.kind = int(qmin), int(qmax), kind
        self._w = None

    def fields(self):
        return dict(zero_point=self.zero_point, scale=self.scale, per_ci=self.per_ci,
                    col_scale=self.col_scale, n_bits=self.n_bits, qmin=self.qmin, qmax=self.qmax,
                    kind=self.kind)

    def forward(self, x=None):
        if self._w is None or self._w.device != self.packed.device:
            self._w = K.pack_decode(self.packed, self.shape, self.zero_point, self.scale,
                                    self.per_ci, self.col_scale, self.n_bits, self.qmin)
        return self._w

    def _apply(self, fn, *args, **kwargs):
        self._w = None
        return super()._apply(fn, *args, **kwargs)


def _layers(qnn):
    return [(n, m) for n, m in qnn.named_modules() if isinstance(m, QuantModule)]


@torch.no_grad()
def export_quantized(qnn, path=None):
    """Packed export of every QuantModule (its weight in its current quantizer's hard
    form, bias, gamma^z/phi^z, activation quantizer).  Returns (tensors, metadata);
    writes a safetensors file when `path` is given."""
    tensors, layers = {}, {}
    for name, m in _layers(qnn):
        what, f = dequant_form(m)
        packed, bad = K.pack_encode(what, f["zero_point"], f["scale"], f["per_ci"], f["col_scale"],
                                    f["n_bits"], f["qmin"], f["qmax"])
        if bad:
            raise ValueError(f"{name}: {bad} weights are not integer codes of the {f['kind']} "
                             "quantizer (soft state?); nothing exported")
        tensors[f"{name}.codes"] = packed
        tensors[f"{name}.zero_point"] = f["zero_point"]
        tensors[f"{name}.scale"] = f["scale"]
        if f["col_scale"] is not None:
            tensors[f"{name}.col_scale"] = f["col_scale"]
        if m.bias is not None:     # the bias the quantized forward adds (quant_layer.py:250)
            tensors[f"{name}.bias"] = m.bias.detach().float().contiguous()
        if not m._affine_is_identity():
            tensors[f"{name}.alpha_out"] = m.alpha_out.detach().contiguous()
            tensors[f"{name}.beta_out"] = m.beta_out.detach().contiguous()
        aq = m.act_quantizer
        act = None
        if not m.disable_act_quant and aq.inited and aq.delta is not None:
            tensors[f"{name}.act_delta"] = aq.delta.detach().reshape(-1).contiguous()
            tensors[f"{name}.act_zero_point"] = aq.zero_point.detach().reshape(-1).contiguous()
            act = dict(n_bits=aq.n_bits, sym=aq.sym)
        layers[name] = dict(shape=list(m.weight.shape), n_bits=f["n_bits"], qmin=f["qmin"],
                            qmax=f["qmax"], per_ci=f["per_ci"], kind=f["kind"], act=act,
                            disable_act_quant=bool(m.disable_act_quant))
    for name, b in qnn.named_modules():
        aq = getattr(b, "act_quantizer", None)
        if name and not isinstance(b, QuantModule) and aq is not None and aq.inited \
                and aq.delta is not None:
            tensors[f"{name}.act_delta"] = aq.delta.detach().reshape(-1).contiguous()
            tensors[f"{name}.act_zero_point"] = aq.zero_point.detach().reshape(-1).contiguous()
            layers[name] = dict(block=True, act=dict(n_bits=aq.n_bits, sym=aq.sym))
    meta = {"format": FORMAT, "layers": json.dumps(layers)}
    if path is not None:
        from safetensors.torch import save_file
        save_file({k: v.contiguous().cpu() for k, v in tensors.items()}, path, metadata=meta)
    return tensors, meta


@torch.no_grad()
def load_quantized(qnn, src, device=None):
    """Install an export into a QuantModel of the same architecture: weights become
    PackedWeight quantizers (decoded on the device), biases / gamma^z / phi^z / act
    quantizer parameters are restored.  `src` is a path or export_quantized's result."""
    if isinstance(src, str):
        from safetensors import safe_open
        with safe_open(src, framework="pt") as fh:
            meta = fh.metadata()
            tensors = {k: fh.get_tensor(k) for k in fh.keys()}
    else:
        tensors, meta = src
    if meta.get("format") != FORMAT:
        raise ValueError(f"not a {FORMAT} export")
    layers = json.loads(meta["layers"])
    device = device or next(qnn.parameters()).device
    t = {k: v.to(device) for k, v in tensors.items()}
    mods = dict(qnn.named_modules())
    for name, info in layers.items():
        m = mods[name]
        if info.get("act") is not None:
            aq = m.act_quantizer
            aq.delta = nn.Parameter(t[f"{name}.act_delta"].reshape(aq.delta.shape if aq.delta is not None
                                                                   else ()).clone())
            aq.zero_point = nn.Parameter(t[f"{name}.act_zero_point"].reshape(aq.delta.shape).clone())
            aq.inited = True
        if info.get("block"):
            continue
        m.disable_act_quant = info["disable_act_quant"]
        m.weight_quantizer = PackedWeight(t[f"{name}.codes"], info["shape"], t[f"{name}.zero_point"],
                                          t[f"{name}.scale"], info["per_ci"],
                                          t.get(f"{name}.col_scale"), info["n_bits"], info["qmin"],
                                          info["qmax"], info["kind"])
        if f"{name}.bias" in t and m.bias is not None:
            m.bias.data.copy_(t[f"{name}.bias"])
        if f"{name}.alpha_out" in t:
            m.alpha_out.data.copy_(t[f"{name}.alpha_out"])
            m.beta_out.data.copy_(t[f"{name}.beta_out"])
    return qnn
