"""Generate the golden fixtures under tests/golden/ by running the REFERENCE on CPU.

This is the only file in the repository that imports /root/reference, and it only
runs in the build container (the reference never travels to the GPU box).  What it
writes is data: seeded inputs and the reference's outputs, as small .npz files.

Loading recipe: stub the absent third-party modules
(icecream, telegram, the git-ignored pretrained CIFAR package, torchvision-backed
data loaders), map hard-coded 'cuda' devices to CPU for the functions that use
them, and import the reference's own quant/ modules unmodified.

Run:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py
"""
import os
import sys
import types

os.environ["PYTHONDONTWRITEBYTECODE"] = "1"
sys.dont_write_bytecode = True

import numpy as np
import torch
import torch.nn as nn

REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, OUT)       # realshape.py: the seeded real-shape cases shared with the tests


# --------------------------------------------------------------------------- stubs
def _install_stubs():
    ic_mod = types.ModuleType("icecream")

    class _IC:
        def configureOutput(self, **k):
            pass

        def disable(self):
            pass

        def __call__(self, *a, **k):
            return a[0] if a else None

    ic_mod.ic = _IC()
    sys.modules["icecream"] = ic_mod

    for name in ["pretrained", "pretrained.PyTorch_CIFAR10",
                 "pretrained.PyTorch_CIFAR10.cifar10_models"]:
        sys.modules[name] = types.ModuleType(name)
    res = types.ModuleType("pretrained.PyTorch_CIFAR10.cifar10_models.resnet")

    class BasicBlockCIFAR(nn.Module):
        pass

    def _absent(*a, **k):
        raise RuntimeError("CIFAR pretrained models are absent")

    res.BasicBlockCIFAR = BasicBlockCIFAR
    res.resnet18 = res.resnet34 = res.resnet50 = _absent
    sys.modules[res.__name__] = res

    tg = types.ModuleType("telegram")
    tg.Bot = object
    sys.modules["telegram"] = tg


def _install_cpu_device_shim():
    """Map 'cuda' device requests to CPU (reference hard-codes them at
    layer_recon_shiftedScale.py:268, block_recon.py:88, layer_recon.py:78)."""
    orig_to = torch.Tensor.to

    def _map(a):
        if isinstance(a, str) and a.startswith("cuda"):
            return "cpu"
        if isinstance(a, torch.device) and a.type == "cuda":
            return torch.device("cpu")
        return a

    def to(self, *args, **kw):
        args = tuple(_map(a) for a in args)
        if "device" in kw:
            kw["device"] = _map(kw["device"])
        return orig_to(self, *args, **kw)

    torch.Tensor.to = to
    orig_device = torch.device

    class _DevMeta(type):
        def __instancecheck__(cls, inst):
            return isinstance(inst, orig_device)

        def __call__(cls, *a, **k):
            if a and isinstance(a[0], str) and a[0].startswith("cuda"):
                a = ("cpu",) + a[1:]
            return orig_device(*a, **k)

    class device(metaclass=_DevMeta):
        pass

    torch.device = device


_install_stubs()
sys.path.insert(0, REF)
from quant.quant_layer import UniformAffineQuantizer, lp_loss, QuantModule  # noqa: E402
from quant.channelQuant import ChannelQuant  # noqa: E402
from quant.channelQuantMSE import ChannelQuantMSE  # noqa: E402
from quant.adaptive_rounding import AdaRoundQuantizer  # noqa: E402
from quant import layer_recon_fused_shiftedScale as LRF  # noqa: E402
from quant import layer_recon_shiftedScale as LRS  # noqa: E402
from quant import block_recon as BR  # noqa: E402
from quant.quant_model import QuantModel  # noqa: E402
from models.resnet import resnet18  # noqa: E402
import myScaledMethods as MSM  # noqa: E402

_install_cpu_device_shim()


def f32(x):
    return np.ascontiguousarray(np.asarray(x, dtype=np.float32))


def t2n(t):
    if t is None:
        return np.zeros(0, np.float32)
    return f32(t.detach().cpu().numpy()).copy()  # never alias a tensor mutated later


def save(name, **arrays):
    path = os.path.join(OUT, name + ".npz")
    np.savez_compressed(path, **{k: np.asarray(v) for k, v in arrays.items()})
    print(f"wrote {path} ({os.path.getsize(path)} B)")


def edge_tensor(g, shape, scale=1.0):
    """Gaussian values plus exact .5 ties and clamp edges after scaling."""
    x = torch.randn(shape, generator=g) * scale
    flat = x.view(-1)
    n = flat.numel()
    k = max(1, n // 16)
    flat[0::16] = (flat[0::16] * 4 / scale).round() * 0.125 * scale  # exact multiples of scale/8
    flat[5::16] = 0.0
    return x


# IEEE special values planted into the *_specials fixtures (after the quantizer's scale was
# initialised on clean data: a NaN in the 'max' init makes the reference's Python round()
# raise): NaN, +-inf, +-0 and the largest finite magnitudes
SPECIALS = [float("nan"), float("inf"), -float("inf"), 0.0, -0.0, 3.0e38, -3.0e38,
            float("nan")]


def special_pos(shape):
    """Fixed, distinct flat positions of SPECIALS: weights ([Co, Ci, ...]) get them in odd
    output channels and in only two input channels (1 and Ci - 2), so that the per-input-
    channel shift logits of the other channels keep finite gradients; other tensors
    (activations) at a fixed stride."""
    shape = tuple(shape)
    n = int(np.prod(shape))
    if len(shape) in (2, 4) and shape[0] >= 4:
        co, ci = shape[0], shape[1]
        cis = [min(1, ci - 1), max(ci - 2, 0)]
        inner = int(np.prod(shape[2:])) if len(shape) == 4 else 1
        pos = []
        for k in range(len(SPECIALS)):
            c, i, t = (2 * k + 1) % co, cis[k % 2], (k * 5) % inner
            p = (c * ci + i) * inner + t
            while p in pos:
                p = (p + 1) % n
            pos.append(p)
        return pos
    pos = []
    k = 0
    while len(pos) < len(SPECIALS):
        p = (k * 37 + 5) % n
        if p not in pos:
            pos.append(p)
        k += 1
    return pos


def with_specials(x):
    y = x.clone()
    flat = y.view(-1)
    for p, v in zip(special_pos(x.shape), SPECIALS):
        flat[p] = v
    return y


# --------------------------------------------------------------------------- K1-K4 UAQ
def gen_uaq():
    g = torch.Generator().manual_seed(1005)
    out = {}
    for bits in (2, 3, 4, 8):
        for sym in (False, True):
            for cw in (False, True):
                for method in ("max", "mse"):
                    tag = f"b{bits}_{'sym' if sym else 'asym'}_{'cw' if cw else 'pt'}_{method}"
                    if not cw and (method == "max" or sym):
                        # per-tensor 'max' and per-tensor symmetric return a Python int
                        # zero_point that nn.Parameter rejects (quant_layer.py:88,140,161):
                        # broken in the reference, so no golden exists for them.
                        continue
                    shape = (12, 5, 3, 3) if cw else (4, 6, 7, 7)
                    x = edge_tensor(g, shape, 0.2 if cw else 1.0)
                    if not cw:
                        x = torch.relu(x) if not sym else x
                    q = UniformAffineQuantizer(n_bits=bits, symmetric=sym, channel_wise=cw,
                                               scale_method=method, leaf_param=not cw,
                                               ch=shape)
                    xr = x.clone().requires_grad_(True)
                    y = q(xr)
                    gy = torch.randn(shape, generator=g)
                    (y * gy).sum().backward()
                    out[tag + "_x"] = t2n(x)
                    out[tag + "_y"] = t2n(y)
                    out[tag + "_delta"] = t2n(q.delta.reshape(-1))
                    out[tag + "_zp"] = t2n(q.zero_point.reshape(-1))
                    rz = q.raw_zero_point
                    out[tag + "_rawzp"] = f32(rz.detach().reshape(-1).numpy() if torch.is_tensor(rz) else [rz])
                    out[tag + "_gy"] = t2n(gy)
                    out[tag + "_gx"] = t2n(xr.grad)
                    out[tag + "_gdelta"] = t2n(q.delta.grad.reshape(-1))
                    out[tag + "_gzp"] = t2n(q.zero_point.grad.reshape(-1))
    # zero-range channel -> delta clamps to 1e-8 (quant_layer.py:136-138)
    x = torch.zeros(3, 4, 3, 3)
    x[1] = 0.5
    q = UniformAffineQuantizer(n_bits=2, channel_wise=True, scale_method="max", ch=x.shape)
    y = q(x)
    out["zero_x"], out["zero_y"] = t2n(x), t2n(y)
    out["zero_delta"], out["zero_zp"] = t2n(q.delta.reshape(-1)), t2n(q.zero_point.reshape(-1))
    save("uaq", **out)


def gen_uaq_specials():
    """UAQ forward + STE backward (quant_layer.py:77-98) and ChannelQuantAct 'none'
    (channelQuantAct.py:36-67) on inputs holding SPECIALS: the scales are initialised on
    the clean tensor, then the quantizer runs on the tensor with the specials planted.
    torch.clamp propagates NaN (the dequant is NaN there), +-inf clamp to the edges, and
    the gradients are whatever the reference's autograd makes of them (NaN in the delta
    sums where a NaN or an inf meets the x/delta path)."""
    from quant.channelQuantAct import ChannelQuantAct
    g = torch.Generator().manual_seed(2718)
    out = {}
    cases = [("b4_asym_pt_mse", 4, False, False, "mse", (4, 6, 7, 7)),
             ("b2_asym_cw_max", 2, False, True, "max", (12, 5, 3, 3)),
             ("b8_asym_cw_max", 8, False, True, "max", (12, 5, 3, 3)),
             ("b4_sym_cw_max", 4, True, True, "max", (12, 5, 3, 3))]
    for tag, bits, sym, cw, method, shape in cases:
        x = edge_tensor(g, shape, 0.2 if cw else 1.0)
        if not cw:
            x = torch.relu(x)
        q = UniformAffineQuantizer(n_bits=bits, symmetric=sym, channel_wise=cw, scale_method=method,
                                   leaf_param=not cw, ch=shape)
        with torch.no_grad():
            q(x)                                   # scale init on the clean tensor
        xs = with_specials(x * 1.5)
        xr = xs.clone().requires_grad_(True)
        y = q(xr)
        gy = torch.randn(shape, generator=g)
        (y * gy).sum().backward()
        out[tag + "_x"] = t2n(xs)
        out[tag + "_y"] = t2n(y)
        out[tag + "_delta"] = t2n(q.delta.reshape(-1))
        out[tag + "_zp"] = t2n(q.zero_point.reshape(-1))
        out[tag + "_gy"] = t2n(gy)
        out[tag + "_gx"] = t2n(xr.grad)
        out[tag + "_gdelta"] = t2n(q.delta.grad.reshape(-1))
        out[tag + "_gzp"] = t2n(q.zero_point.grad.reshape(-1))
        if tag == "b4_asym_pt_mse":
            # ChannelQuantAct 'none' on the same tensor (no STE: torch.round)
            for k, sc in enumerate((1.0, 0.5)):
                ca = ChannelQuantAct(uaq=q, shiftTarget=[1.0, 0.5])
                ca.shiftedScale = sc
                q.delta.grad = None
                q.zero_point.grad = None
                xr = xs.clone().requires_grad_(True)
                ya = ca(xr)
                (ya * gy).sum().backward()
                out[f"act_s{k}_scale"] = np.array([sc], np.float64)
                out[f"act_s{k}_y"] = t2n(ya)
                out[f"act_s{k}_gdelta"] = t2n(q.delta.grad.reshape(-1))
                out[f"act_s{k}_gzp"] = t2n(q.zero_point.grad.reshape(-1))
    save("uaq_specials", **out)


def gen_init_specials():
    """init_quantization_scale (quant_layer.py:100-166) on inputs holding SPECIALS BEFORE the
    init.  Per case: status 0 = the reference returns a usable scale (delta / zp / raw_zp
    recorded per row), 1 = it raises (its exception's type name recorded: round(nan) is a
    ValueError at :140; a None delta assigned into a channel's slot a TypeError at :114),
    2 = it returns delta None (per-tensor 'mse' when no candidate scores below 1e10,
    :147-162), which the quantizer cannot use."""
    g = torch.Generator().manual_seed(31337)
    out, names = {}, []
    shape = (6, 5, 3, 3)
    plants = {"nan": float("nan"), "pinf": float("inf"), "ninf": -float("inf"),
              "big": 3.0e38, "const": None, "zero": None}
    for method in ("max", "mse"):
        for cw in (True, False):
            for sym in (False, True):
                for pname, val in plants.items():
                    x = edge_tensor(g, shape, 0.2)
                    if not cw and not sym:
                        x = torch.relu(x)
                    if pname == "const":
                        x[3] = 0.375
                    elif pname == "zero":
                        x[3] = 0.0
                    else:
                        x[3, 2, 1, 0] = val
                    tag = f"{method}_{'cw' if cw else 'pt'}_{'sym' if sym else 'asym'}_{pname}"
                    q = UniformAffineQuantizer(n_bits=4, symmetric=sym, channel_wise=cw,
                                               scale_method=method, ch=shape)
                    out[tag + "_x"] = t2n(x)
                    try:
                        d, z, r = q.init_quantization_scale(x.clone(), channel_wise=cw)
                    except Exception as e:  # the reference's own failure, recorded as data
                        out[tag + "_status"] = np.array([1], np.int32)
                        out[tag + "_exc"] = np.array([type(e).__name__])
                        names.append(tag)
                        continue
                    if d is None:
                        out[tag + "_status"] = np.array([2], np.int32)
                        names.append(tag)
                        continue
                    out[tag + "_status"] = np.array([0], np.int32)
                    for k, v in (("delta", d), ("zp", z), ("rawzp", r)):
                        out[tag + "_" + k] = f32(v.detach().reshape(-1).numpy()
                                                 if torch.is_tensor(v) else [v])
                    names.append(tag)
    out["cases"] = np.array(names)
    save("init_specials", **out)


# --------------------------------------------------------------------------- K5-K9 ChannelQuant
def _mk_uaq(w, bits=2, method="max"):
    q = UniformAffineQuantizer(n_bits=bits, channel_wise=True, scale_method=method, ch=w.shape)
    q(w)
    return q


def gen_channelquant(specials=False):
    """specials=True: the same cases with SPECIALS planted into the weight AFTER the UAQ
    scale init (init_v_beta, every mode and the AdaRound phase then see them), written to
    channelquant_specials.npz with the same keys."""
    g = torch.Generator().manual_seed(1005)
    out = {}
    shapes = {"conv": (8, 6, 3, 3), "fc": (10, 12), "dw": (6, 1, 3, 3)}
    shift = [31 / 32, 33 / 32, 1.0]
    for name, shape in shapes.items():
        for bits in (2, 4):
            tag = f"{name}_b{bits}"
            w = torch.randn(shape, generator=g) * 0.05
            uaq = _mk_uaq(w, bits)
            w_clean = w
            if specials:
                w = with_specials(w)
            cq = ChannelQuant(1.0, uaq=uaq, weight_tensor=w, shiftTarget=shift, name=tag)
            cq.init_v_beta(w.clone())
            cq.opt_mode = "adaShift"
            out[tag + "_w"] = t2n(w)
            out[tag + "_delta"] = t2n(cq.delta.reshape(-1))
            out[tag + "_zp"] = t2n(cq.zero_point.reshape(-1))
            out[tag + "_xq"] = np.stack([t2n(t) for t in cq.x_q])
            out[tag + "_alpha0"] = t2n(cq.alpha)
            out[tag + "_beta"] = t2n(cq.beta)
            # perturb alpha so soft targets are not all at init
            with torch.no_grad():
                cq.alpha.add_(torch.randn(cq.alpha.shape, generator=g) * 0.5)
            out[tag + "_alpha"] = t2n(cq.alpha)
            gy = torch.randn(shape, generator=g)
            out[tag + "_gy"] = t2n(gy)
            for hard_t, hard_r in ((False, False), (True, True), (False, True), (True, False)):
                cq.hard_targets, cq.hard_round = hard_t, hard_r
                cq.alpha.grad = None
                cq.beta.grad = None
                y = cq(w)
                k = f"{tag}_t{int(hard_t)}r{int(hard_r)}"
                out[k + "_y"] = t2n(y)
                if y.requires_grad:
                    (y * gy).sum().backward()
                    out[k + "_galpha"] = t2n(cq.alpha.grad) if cq.alpha.grad is not None else np.zeros(0, np.float32)
                    out[k + "_gbeta"] = t2n(cq.beta.grad) if cq.beta.grad is not None else np.zeros(0, np.float32)
            cq.hard_targets = cq.hard_round = False
            out[tag + "_p"] = t2n(cq.get_sig_soft_targets())
            out[tag + "_h"] = t2n(cq.get_soft_round())
            out[tag + "_delta_sel"] = t2n(cq.get_delta())

            # learned_hard_sigmoid path (init_v, channelQuant.py:201-213)
            uaq2 = _mk_uaq(w_clean, bits)
            cq2 = ChannelQuant(1.0, uaq=uaq2, weight_tensor=w, shiftTarget=shift, name=tag)
            cq2.init_v(w.clone())
            out[tag + "_lhs_xq"] = np.stack([t2n(t) for t in cq2.x_q])
            out[tag + "_lhs_alpha0"] = t2n(cq2.alpha)
            with torch.no_grad():
                cq2.alpha.add_(torch.randn(cq2.alpha.shape, generator=g) * 0.5)
            out[tag + "_lhs_alpha"] = t2n(cq2.alpha)
            for hard_t in (False, True):
                cq2.hard_targets = hard_t
                cq2.alpha.grad = None
                y = cq2(w)
                out[f"{tag}_lhs_t{int(hard_t)}_y"] = t2n(y)
                if y.requires_grad:
                    (y * gy).sum().backward()
                    out[f"{tag}_lhs_t{int(hard_t)}_galpha"] = t2n(cq2.alpha.grad)
            # adaround phase (layer_recon_shiftedScale.py:270-276): update_delta + init_beta
            cq2.hard_targets = False
            cq2.update_delta()
            cq2.init_beta(w.clone())
            cq2.opt_mode = "adaround"
            out[tag + "_ar_delta"] = t2n(cq2.delta)
            out[tag + "_ar_beta0"] = t2n(cq2.beta)
            with torch.no_grad():
                cq2.beta.add_(torch.randn(cq2.beta.shape, generator=g) * 0.5)
            out[tag + "_ar_beta"] = t2n(cq2.beta)
            for hard_r in (False, True):
                cq2.hard_round = hard_r
                cq2.beta.grad = None
                y = cq2(w)
                out[f"{tag}_ar_r{int(hard_r)}_y"] = t2n(y)
                if y.requires_grad:
                    (y * gy).sum().backward()
                    out[f"{tag}_ar_r{int(hard_r)}_gbeta"] = t2n(cq2.beta.grad)
            cq2.opt_mode = "none"
            out[tag + "_none_y"] = t2n(cq2(w))
    save("channelquant_specials" if specials else "channelquant", **out)


def gen_adaround(specials=False):
    """specials=True: SPECIALS planted into the weight after the UAQ scale init
    (adaround_specials.npz, same keys)."""
    g = torch.Generator().manual_seed(1005)
    out = {}
    for name, shape in {"conv": (8, 6, 3, 3), "fc": (10, 12)}.items():
        w = torch.randn(shape, generator=g) * 0.05
        uaq = _mk_uaq(w, 2)
        if specials:
            w = with_specials(w)
        ar = AdaRoundQuantizer(uaq=uaq, round_mode="learned_hard_sigmoid", weight_tensor=w)
        out[name + "_w"] = t2n(w)
        out[name + "_delta"] = t2n(ar.delta.reshape(-1))
        out[name + "_zp"] = t2n(ar.zero_point.reshape(-1))
        out[name + "_alpha0"] = t2n(ar.alpha)
        with torch.no_grad():
            ar.alpha.add_(torch.randn(shape, generator=g) * 0.5)
        out[name + "_alpha"] = t2n(ar.alpha)
        gy = torch.randn(shape, generator=g)
        out[name + "_gy"] = t2n(gy)
        for soft in (True, False):
            ar.soft_targets = soft
            ar.alpha.grad = None
            y = ar(w)
            out[f"{name}_s{int(soft)}_y"] = t2n(y)
            if y.requires_grad:
                (y * gy).sum().backward()
                out[f"{name}_s{int(soft)}_galpha"] = t2n(ar.alpha.grad)
        out[name + "_h"] = t2n(ar.get_soft_targets())
    save("adaround_specials" if specials else "adaround", **out)


# --------------------------------------------------------------------------- K10
def gen_inpscale():
    g = torch.Generator().manual_seed(1005)
    out = {}
    for bits in (2, 4):
        w = torch.randn(16, 8, 3, 3, generator=g) * 0.05
        for level in (1, 2, 8, 64):
            for thr in (1.0, 2.0):
                tag = f"b{bits}_l{level}_t{int(thr)}"
                uaq = _mk_uaq(w, bits)
                m = ChannelQuantMSE(1.0, uaq=uaq, weight_tensor=w, shiftTarget=[1.0], opt_mode="max",
                                    level=level, threshold=thr, name=tag)
                m.init_scale(w)
                out[tag + "_inp"] = t2n(m.inp_scale)
                out[tag + "_y"] = t2n(m(w))
        out[f"b{bits}_w"] = t2n(w)
        out[f"b{bits}_delta"] = t2n(uaq.delta.reshape(-1))
        out[f"b{bits}_rawzp"] = t2n(uaq.raw_zero_point.reshape(-1))
    # FC variant
    w = torch.randn(10, 12, generator=g) * 0.05
    uaq = _mk_uaq(w, 2)
    m = ChannelQuantMSE(1.0, uaq=uaq, weight_tensor=w, shiftTarget=[1.0], opt_mode="max", level=8,
                        threshold=2.0, name="fc")
    m.init_scale(w)
    out["fc_w"], out["fc_inp"], out["fc_y"] = t2n(w), t2n(m.inp_scale), t2n(m(w))
    out["fc_delta"], out["fc_rawzp"] = t2n(uaq.delta.reshape(-1)), t2n(uaq.raw_zero_point.reshape(-1))
    save("inpscale", **out)


# --------------------------------------------------------------------------- K11/K12
def gen_loss():
    g = torch.Generator().manual_seed(1005)
    out = {}
    pred = torch.randn(4, 6, 5, 5, generator=g)
    tgt = torch.randn(4, 6, 5, 5, generator=g)
    out["pred"], out["tgt"] = t2n(pred), t2n(tgt)
    for p in (1.0, 2.0, 2.4):
        for red in ("none", "all"):
            pr = pred.clone().requires_grad_(True)
            l = lp_loss(pr, tgt, p=p, reduction=red)
            l.backward()
            out[f"p{p}_{red}_loss"] = f32([l.item()])
            out[f"p{p}_{red}_grad"] = t2n(pr.grad)
    # regularizers (layer_recon_fused_shiftedScale.py:277-282, layer_recon_shiftedScale.py:393,
    # block_recon.py:171-174)
    v = torch.randn(6, 3, generator=g) * 2
    beta = torch.randn(8, 6, 3, 3, generator=g) * 2
    out["reg_alpha"], out["reg_beta"] = t2n(v), t2n(beta)
    gam, zet = -0.1, 1.1
    for b in (0.0, 20.0, 11.3, 2.0):
        a = v.clone().requires_grad_(True)
        pS = torch.clamp(torch.softmax(a, dim=-1) * (zet - gam) + gam, 0, 1)
        lS = 0.1 * (1 - ((pS - .5).abs() * 2).pow(b)).sum()
        lS.backward()
        out[f"regS_b{b}_loss"], out[f"regS_b{b}_grad"] = f32([lS.item()]), t2n(a.grad)
        bb = beta.clone().requires_grad_(True)
        hR = torch.clamp(torch.sigmoid(bb) * (zet - gam) + gam, 0, 1)
        lR = 0.01 * (1 - ((hR - .5).abs() * 2).pow(b)).sum()
        lR.backward()
        out[f"regR_b{b}_loss"], out[f"regR_b{b}_grad"] = f32([lR.item()]), t2n(bb.grad)
    a = v.clone().requires_grad_(True)
    pS = torch.clamp(torch.softmax(a, dim=-1) * (zet - gam) + gam, 0, 1)
    lE = 0.1 * (-torch.sum(pS * torch.log(pS + 1e-10)))
    lE.backward()
    out["regE_loss"], out["regE_grad"] = f32([lE.item()]), t2n(a.grad)
    # schedules
    ts = np.arange(0, 101, dtype=np.int64)
    fused = LRF.FusedLinearTempDecayShift(100, rel_start_decay=0.2, start_b=20, end_b=2)
    fused_s = LRF.FusedLinearTempDecayShift(100 * 3 / 4, rel_start_decay=0.2, start_b=20, end_b=2)
    lin = BR.LinearTempDecay(100, rel_start_decay=0.2, start_b=20, end_b=2)
    lsh = LRS.LinearTempDecayShift(100, rel_start_decay=0.2, start_b=20, end_b=2)
    out["sched_t"] = ts
    out["sched_fused"] = np.array([fused(t) for t in ts], np.float64)
    out["sched_fused_shift"] = np.array([fused_s(t) for t in ts], np.float64)
    out["sched_lin"] = np.array([lin(t) for t in ts], np.float64)
    out["sched_lsh"] = np.array([lsh(t) for t in ts], np.float64)
    save("loss", **out)


# --------------------------------------------------------------------------- loop golden
def _tiny_net():
    """stem conv -> BN -> ReLU -> BasicBlock(16->32, stride 2, downsample) -> pool -> fc.
    Small enough that the block's weights and features fit a sub-MB fixture; built from
    the reference's own BasicBlock so QuantModel wraps it as a QuantBasicBlock."""
    from models.resnet import BasicBlock
    torch.manual_seed(1005)
    ds = nn.Sequential(nn.Conv2d(16, 32, 1, stride=2, bias=False), nn.BatchNorm2d(32))
    net = nn.Sequential(nn.Conv2d(3, 16, 3, padding=1, bias=False), nn.BatchNorm2d(16), nn.ReLU(),
                        BasicBlock(16, 32, stride=2, downsample=ds, norm_layer=nn.BatchNorm2d),
                        nn.AdaptiveAvgPool2d(1), nn.Flatten(), nn.Linear(32, 10))
    g = torch.Generator().manual_seed(7)
    for m in net.modules():
        if isinstance(m, nn.Conv2d):
            nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
        if isinstance(m, nn.BatchNorm2d):  # non-trivial folded statistics
            m.running_mean.copy_(torch.randn(m.num_features, generator=g) * 0.1)
            m.running_var.copy_(torch.rand(m.num_features, generator=g) + 0.5)
            m.weight.data.copy_(torch.rand(m.num_features, generator=g) + 0.5)
            m.bias.data.copy_(torch.randn(m.num_features, generator=g) * 0.1)
    return net.eval()


def _build_tiny_qnn(bits_w=2, bits_a=4):
    wq = {"n_bits": bits_w, "channel_wise": True, "scale_method": "max", "tune_delta_zero": False,
          "symmetric": False}
    aq = {"n_bits": bits_a, "channel_wise": False, "scale_method": "mse", "tune_delta_zero": False,
          "leaf_param": True, "symmetric": False}
    qnn = QuantModel(model=_tiny_net(), weight_quant_params=wq, act_quant_params=aq)
    qnn.eval()
    qnn.set_first_last_layer_to_8bit()
    return qnn


BLOCK = ".model.3"
CONVS = ("conv1", "conv2", "downsample")


def _cache(qnn, names, cali, bs):
    MSM.set_cache_state(qnn, names, prv_name="", state="if")
    with torch.no_grad():
        for i in range(len(cali) // bs):
            qnn(cali[i * bs:(i + 1) * bs])
    qnn.store_quantization_state()
    qnn.set_quant_state(False, False)
    MSM.set_cache_state(qnn, names, prv_name="", state="of")
    with torch.no_grad():
        for i in range(len(cali) // bs):
            qnn(cali[i * bs:(i + 1) * bs])
    qnn.restore_quantization_state()
    MSM.set_cache_state(qnn, names, prv_name="", state="none")


class _Spy:
    """Records randperm draws and per-iteration loss values of a reference loop."""

    def __init__(self, loss_cls):
        self.loss_cls, self.perms, self.rec = loss_cls, [], []

    def __enter__(self):
        self.orig_call, self.orig_rp = self.loss_cls.__call__, torch.randperm
        spy = self

        def call(lf, pred, tgt, grad=None):
            r = spy.orig_call(lf, pred, tgt, grad)
            rl = getattr(lf, "rec_loss", 0.0)
            spy.rec.append((float(rl) if not isinstance(rl, str) else float("nan"), float(r.item())))
            return r

        def rp(n, *a, **k):
            r = spy.orig_rp(n, *a, **k)
            spy.perms.append(r.clone())
            return r

        self.loss_cls.__call__ = call
        torch.randperm = rp
        return self

    def __exit__(self, *exc):
        self.loss_cls.__call__ = self.orig_call
        torch.randperm = self.orig_rp


class _GradSpy:
    """Records, at the chosen optimizer step counts (counted over every torch.optim.Adam
    step taken inside the context), each optimised parameter's value before the step and
    the gradient the reference's backward handed to it."""

    def __init__(self, at, truth=None):
        self.at, self.n, self.rec, self.truth, self.rec64 = set(at), 0, {}, truth, {}

    def __enter__(self):
        self.orig = torch.optim.Adam.step
        spy = self

        def step(opt, *a, **k):
            if spy.n in spy.at:
                ps = [p for grp in opt.param_groups for p in grp["params"]]
                spy.rec[spy.n] = ([t2n(p) for p in ps], [t2n(p.grad) for p in ps])
                if spy.truth is not None:
                    spy.rec64[spy.n] = spy.truth(spy.n)
            spy.n += 1
            return spy.orig(opt, *a, **k)

        torch.optim.Adam.step = step
        return self

    def __exit__(self, *exc):
        torch.optim.Adam.step = self.orig

    def dump(self, out, prefix=""):
        """Full parameters and gradients (small tensors only)."""
        for s, (ps, gs) in sorted(self.rec.items()):
            for j, (p, g) in enumerate(zip(ps, gs)):
                out[f"{prefix}gs{s}_p{j}"] = p
                out[f"{prefix}gs{s}_g{j}"] = g
            for j, t in enumerate(self.rec64.get(s, [])):
                out[f"{prefix}gs{s}_t{j}"] = t
        out[prefix + "grad_steps"] = np.array(sorted(self.rec), np.int64)


def _to64(mod):
    """`mod` in float64: parameters and buffers (.double()) and every float tensor held as
    a plain attribute or in a list attribute (ChannelQuant's x_q, org_weight, caches)."""
    mod.double()
    for m in mod.modules():
        for k, v in list(vars(m).items()):
            if isinstance(v, nn.Parameter):
                continue
            if isinstance(v, torch.Tensor) and v.is_floating_point():
                setattr(m, k, v.detach().double())
            elif isinstance(v, list) and v and all(isinstance(t, torch.Tensor) for t in v):
                setattr(m, k, [t.detach().double() if t.is_floating_point() else t for t in v])
    return mod


def _layer_truth(layer, spy, lmda, iters, adaround, batch_size=32):
    """As _fused_truth, for layer_recon_shiftedScale's loop (ScaleLossFunction): the
    gradient of the shift logits alpha (shift phase) or of AdaRound's beta (adaround
    phase) in float64 at the fp32 run's parameters of iteration `step`."""
    import copy

    def truth(step):
        l64 = _to64(copy.deepcopy(layer))
        q = l64.weight_quantizer
        p = q.beta if adaround else q.alpha
        p.grad = None
        lf = LRS.ScaleLossFunction(l64, round_loss="relaxation", lmda=lmda, max_count=iters,
                                   b_range=(20, 2), decay_start=0, warmup=0.2, p=2.0,
                                   adaround=adaround)
        lf.count = step
        perm = spy.perms[-1][:batch_size]
        inp = torch.cat(l64.cached_inp_features)[perm]
        tgt = torch.cat(l64.cached_out_features)[perm]
        spy.orig_call(lf, l64(inp), tgt).backward()
        return [np.asarray(p.grad.detach().numpy(), np.float64).copy()]
    return truth


def _fused_truth(block, spy, lmda, iters, batch_size=32, bias_cal=False):
    """The reference's own fused-loop gradient of iteration `step`, evaluated in float64 at
    the parameters the fp32 run holds there (same batch, same loss schedule): the exact
    gradient both fp32 implementations approximate.  bias_cal: also gamma^z / phi^z, in the
    optimizer's order (alpha, alpha_out, beta_out per QuantModule)."""
    import copy

    def truth(step):
        b64 = _to64(copy.deepcopy(block))
        mods = [m for m in b64.modules() if isinstance(m, QuantModule)]
        qs = [m.weight_quantizer for m in mods]
        for m in mods:
            m.weight_quantizer.alpha.grad = None
            m.alpha_out.grad = m.beta_out.grad = None
        lf = LRF.FusedScaleLossFunction(b64, qs, round_loss="relaxation", lmda=lmda, max_count=iters,
                                        b_range=(20, 2), decay_start=0, warmup=0.2, p=2.0)
        lf.count = step
        perm = spy.perms[-1][:batch_size]
        inp = torch.cat(b64.cached_inp_features)[perm]
        tgt = torch.cat(b64.cached_out_features)[perm]
        spy.orig_call(lf, b64(inp), tgt).backward()
        ts = []
        for m in mods:
            ts.append(m.weight_quantizer.alpha.grad)
            if bias_cal:
                ts += [m.alpha_out.grad, m.beta_out.grad]
        return [np.asarray(t.detach().numpy(), np.float64).copy() for t in ts]
    return truth


class _BiasCalAdam:
    """Oracle-side shim for --bias_cal (README.md:20,33): the reference's own intent, the
    commented-out `opt_params += [module.alpha_out]` / `[module.beta_out]` lines right after
    each shift logit (layer_recon_fused_shiftedScale.py:65-68; the parameters:
    quant_layer.py:231-238, applied at :258-259).  Inside the context the Adam the loop
    builds (:73) also holds, after each QuantModule's alpha, that module's gamma^z and
    phi^z -- nothing else of the reference changes."""

    def __init__(self, block):
        self.mods = [m for m in block.modules() if isinstance(m, QuantModule)]

    def __enter__(self):
        self.orig = torch.optim.Adam
        mods, orig = self.mods, self.orig

        class Adam(orig):
            def __init__(self, params, *a, **k):
                out = []
                for p in list(params):
                    out.append(p)
                    for m in mods:
                        if m.weight_quantizer.alpha is p:
                            out += [m.alpha_out, m.beta_out]
                super().__init__(out, *a, **k)

        torch.optim.Adam = Adam
        return self

    def __exit__(self, *exc):
        torch.optim.Adam = self.orig


def _dump_block(out, block, prefix=""):
    for n in CONVS:
        m = getattr(block, n)
        out[prefix + n + "_w"] = t2n(m.org_weight)
        out[prefix + n + "_b"] = t2n(m.org_bias)


def gen_recon_fused(iters=30, n_cali=16, res=16, bias_cal=False):
    """block_recon_fused_shiftedScale on the tiny net's BasicBlock.  bias_cal=True:
    under _BiasCalAdam (gamma^z / phi^z learned too) -> recon_fused_biascal.npz, with their
    values / gradients in the gs<step>_p/g/t records and their final values."""
    qnn = _build_tiny_qnn()
    torch.manual_seed(1005)
    cali = torch.randn(n_cali, 3, res, res)
    qnn.set_quant_state(True, False)
    with torch.no_grad():
        qnn(cali[:8])
    shift = [31 / 32, 33 / 32, 1.0]
    MSM.build_ShiftedChannelQuant(qnn, [BLOCK], "", shiftTarget=shift, skipShiftLayer=[])
    qnn.set_quant_state(False, False)
    _cache(qnn, [BLOCK], cali, 8)
    MSM.set_quant_state_block(qnn, [BLOCK], "", True)
    block = qnn.model[3]
    out = {}
    _dump_block(out, block)
    for n in CONVS:
        q = getattr(block, n).weight_quantizer
        out[n + "_delta"] = t2n(q.delta.reshape(-1))
        out[n + "_zp"] = t2n(q.zero_point.reshape(-1))
    out["cached_inp"] = t2n(torch.cat(block.cached_inp_features))
    out["cached_out"] = t2n(torch.cat(block.cached_out_features))
    torch.manual_seed(1005)
    import contextlib
    with _Spy(LRF.FusedScaleLossFunction) as spy, \
            (_BiasCalAdam(block) if bias_cal else contextlib.nullcontext()):
        with _GradSpy((0, 5, 20, iters - 1),
                      _fused_truth(block, spy, (0.01, 0.1), iters, bias_cal=bias_cal)) as gspy:
            res_loss = LRF.block_recon_fused_shiftedScale(block, iters, (0.01, 0.1), qnn, None)
    gspy.dump(out)
    out["perms"] = np.stack([p.numpy() for p in spy.perms]).astype(np.int64)
    out["rec_loss"] = np.array([r[0] for r in spy.rec], np.float64)
    out["total_loss"] = np.array([r[1] for r in spy.rec], np.float64)
    out["final_losses"] = np.array(res_loss, np.float64)
    for n in CONVS:
        m = getattr(block, n)
        q = m.weight_quantizer
        out[n + "_alpha"] = t2n(q.alpha)
        out[n + "_beta0"] = t2n(q.beta)  # beta is never optimised in the fused loop
        out[n + "_gamma"] = t2n(m.alpha_out)
        out[n + "_phi"] = t2n(m.beta_out)
        with torch.no_grad():
            out[n + "_what_hard"] = t2n(q(m.weight))
    out["iters"] = np.array([iters])
    save("recon_fused_biascal" if bias_cal else "recon_fused", **out)


def gen_recon_layer_shift(iters=20, n_cali=16, res=16):
    """layer_recon_shiftedScale: shift phase then adaround phase on one conv."""
    qnn = _build_tiny_qnn(bits_w=4, bits_a=8)
    torch.manual_seed(1005)
    cali = torch.randn(n_cali, 3, res, res)
    qnn.set_quant_state(True, False)
    with torch.no_grad():
        qnn(cali[:8])
    layer = BLOCK + ".conv1"
    MSM.build_ShiftedChannelQuant(qnn, [BLOCK], "", shiftTarget=[31 / 32, 33 / 32, 1.0],
                                  skipShiftLayer=[])
    qnn.set_quant_state(False, False)
    _cache(qnn, [layer], cali, 8)
    m = qnn.model[3].conv1
    m.use_weight_quant = True
    out = {"w": t2n(m.org_weight), "b": t2n(m.org_bias),
           "delta": t2n(m.weight_quantizer.delta.reshape(-1)),
           "zp": t2n(m.weight_quantizer.zero_point.reshape(-1)),
           "cached_inp": t2n(torch.cat(m.cached_inp_features)),
           "cached_out": t2n(torch.cat(m.cached_out_features))}
    torch.manual_seed(1005)
    with _Spy(LRS.ScaleLossFunction) as spy, \
            _GradSpy((0, 5, iters - 1), _layer_truth(m, spy, 0.1, iters, False)) as gspy:
        l1 = LRS.layer_recon_shiftedScale(m, iters, 0.1, qnn, None)
    gspy.dump(out, "shift_")
    out["shift_perms"] = np.stack([p.numpy() for p in spy.perms]).astype(np.int64)
    out["shift_total_loss"] = np.array([r[1] for r in spy.rec], np.float64)
    out["shift_rec_loss"] = np.array([r[0] for r in spy.rec], np.float64)
    out["shift_final"] = np.array(l1, np.float64)
    out["shift_alpha"] = t2n(m.weight_quantizer.alpha)
    out["shift_xq"] = np.stack([t2n(t) for t in m.weight_quantizer.x_q])
    m.weight_quantizer.hard_targets = False
    with _Spy(LRS.ScaleLossFunction) as spy, \
            _GradSpy((0, 5, iters - 1), _layer_truth(m, spy, 0.01, iters, True)) as gspy:
        l2 = LRS.layer_recon_shiftedScale(m, iters, 0.01, qnn, None, adaround=True)
    gspy.dump(out, "ar_")
    out["ar_perms"] = np.stack([p.numpy() for p in spy.perms]).astype(np.int64)
    out["ar_total_loss"] = np.array([r[1] for r in spy.rec], np.float64)
    out["ar_rec_loss"] = np.array([r[0] for r in spy.rec], np.float64)
    out["ar_final"] = np.array(l2, np.float64)
    out["ar_delta"] = t2n(m.weight_quantizer.delta)
    out["ar_beta"] = t2n(m.weight_quantizer.beta)
    with torch.no_grad():
        out["ar_what"] = t2n(m.weight_quantizer(m.weight))
    out["iters"] = np.array([iters])
    save("recon_layer_shift", **out)


def gen_recon_brecq(iters=10, n_cali=16, res=16, name="recon_brecq", affine=False):
    """BRECQ block_reconstruction (AdaRound weights), then the act-delta (LSQ) branch.
    name="recon_brecq_long": the same at a long horizon (iters=400), where the AdaRound b
    schedule (block_recon.py:185-202) reaches its end and the act phase's cosine LR decays to
    zero (Brecq/main_imagenet.py's CosineAnnealingLR(T_max=iters)).  affine=True
    ("recon_brecq_affine"): the block's QuantModules carry seeded non-identity gamma^z /
    phi^z (alpha_out / beta_out, quant_layer.py:231-238, applied at :258-259) -- the state the
    act phase meets after a --bias_cal weight phase."""
    qnn = _build_tiny_qnn()
    torch.manual_seed(1005)
    cali = torch.randn(n_cali, 3, res, res)
    qnn.set_quant_state(True, False)
    with torch.no_grad():
        qnn(cali[:8])
    block = qnn.model[3]
    out = {"cali": t2n(cali)}
    if affine:
        gen = torch.Generator().manual_seed(7)
        for n in CONVS:
            m = getattr(block, n)
            with torch.no_grad():
                m.alpha_out.copy_(1 + 0.05 * torch.randn(m.alpha_out.shape, generator=gen))
                m.beta_out.copy_(0.02 * torch.randn(m.beta_out.shape, generator=gen))
            out[n + "_gamma"] = t2n(m.alpha_out)
            out[n + "_phi"] = t2n(m.beta_out)
    _dump_block(out, block)
    qms = [m for m in qnn.modules() if isinstance(m, QuantModule)]
    for k, m in enumerate(qms):   # whole-network state: asym capture runs the stem too
        out[f"qm{k}_w"], out[f"qm{k}_b"] = t2n(m.org_weight), t2n(m.org_bias)
        out[f"qm{k}_delta"] = t2n(m.weight_quantizer.delta.reshape(-1))
        out[f"qm{k}_zp"] = t2n(m.weight_quantizer.zero_point.reshape(-1))
        out[f"qm{k}_bits"] = np.array([m.weight_quantizer.n_bits])
    for n in CONVS:
        q = getattr(block, n).weight_quantizer
        out[n + "_delta"] = t2n(q.delta.reshape(-1))
        out[n + "_zp"] = t2n(q.zero_point.reshape(-1))
    torch.manual_seed(1005)
    with _Spy(BR.LossFunction) as spy:
        BR.block_reconstruction(qnn, block, cali, batch_size=8, iters=iters, weight=0.01,
                                asym=True, b_range=(20, 2), warmup=0.2, act_quant=False, opt_mode="mse")
    out["w_perms"] = np.stack([p.numpy() for p in spy.perms]).astype(np.int64)
    out["w_total_loss"] = np.array([r[1] for r in spy.rec], np.float64)
    for n in CONVS:
        m = getattr(block, n)
        out[n + "_alpha"] = t2n(m.weight_quantizer.alpha)
        with torch.no_grad():
            out[n + "_what_hard"] = t2n(m.weight_quantizer(m.weight))
    # act phase (Brecq/main_imagenet.py:231-241): act-delta init on 8 samples, then LSQ recon
    qnn.set_quant_state(True, True)
    with torch.no_grad():
        qnn(cali[:8])
    qnn.disable_network_output_quantization()
    aqs = [block.act_quantizer] + [m.act_quantizer for m in (block.conv1, block.conv2, block.downsample)
                                   if m.act_quantizer.delta is not None]
    out["a_delta0"] = np.array([float(q.delta) for q in aqs], np.float32)
    out["a_zp0"] = np.array([float(q.zero_point) for q in aqs], np.float32)
    # act_truth > 0: the first act_truth act iterations' loss also in float64 at the fp32 run's
    # own state and batch -- the reference's distance from exact arithmetic, activation
    # rounding decisions included (recon_brecq_long)
    act_truth = 20 if name == "recon_brecq_long" else 0
    cache, l64s = {}, []
    orig_save = BR.save_inp_oup_data

    def save_io(*a, **k):
        r = orig_save(*a, **k)
        cache["inp"], cache["out"] = r
        return r

    torch.manual_seed(1005)
    BR.save_inp_oup_data = save_io
    try:
        with _Spy(BR.LossFunction) as spy:
            if act_truth:
                orig_call = BR.LossFunction.__call__

                def call64(lf, pred, tgt, grad=None):
                    r = orig_call(lf, pred, tgt, grad)
                    if len(l64s) < act_truth:
                        import copy
                        b64 = _to64(copy.deepcopy(block))
                        perm = spy.perms[-1][:8]
                        with torch.no_grad():
                            y64 = b64(cache["inp"][perm].double())
                            l64s.append(float(BR.lp_loss(y64, cache["out"][perm].double(), p=2.4)))
                    return r
                BR.LossFunction.__call__ = call64
            try:
                BR.block_reconstruction(qnn, block, cali, batch_size=8, iters=iters, act_quant=True,
                                        opt_mode="mse", lr=4e-4, p=2.4)
            finally:
                if act_truth:
                    BR.LossFunction.__call__ = orig_call
    finally:
        BR.save_inp_oup_data = orig_save
    out["a_perms"] = np.stack([p.numpy() for p in spy.perms]).astype(np.int64)
    out["a_total_loss"] = np.array([r[1] for r in spy.rec], np.float64)
    if act_truth:
        out["a_total_loss64"] = np.array(l64s, np.float64)
    out["a_delta"] = np.array([float(q.delta) for q in aqs], np.float32)
    out["iters"] = np.array([iters])
    save(name, **out)


def gen_recon_layer_brecq(iters=10, n_cali=16, res=16):
    """a22, BRECQ's per-layer path: layer_reconstruction (quant/layer_recon.py:10-104, its own
    LossFunction :107-170) as Brecq/main_imagenet.py's recon_model calls it for a
    QuantModule, on the tiny net's block conv1 (3x3 conv, 2-bit) and on its fc (Linear,
    8-bit last layer), in that order (the fc's captured input then carries conv1's finished
    hard rounding): the AdaRound weight phase, then after the act-delta init the act phase
    (Adam lr 4e-4 on the act delta, cosine LR, p = 2.4).  The fc's act quantizer is the
    network output's, disabled (disable_network_output_quantization), so its delta reaches
    no output: no gradient, no Adam step -- only the loss values are recorded."""
    from quant import layer_recon as LR
    qnn = _build_tiny_qnn()
    torch.manual_seed(1005)
    cali = torch.randn(n_cali, 3, res, res)
    qnn.set_quant_state(True, False)
    with torch.no_grad():
        qnn(cali[:8])
    out = {"cali": t2n(cali)}
    _dump_qms(out, qnn, "")
    layers = [("conv", qnn.model[3].conv1), ("fc", qnn.model[6])]
    assert isinstance(layers[1][1], QuantModule) and layers[1][1].weight.dim() == 2
    for tag, layer in layers:
        torch.manual_seed(1005)
        with _Spy(LR.LossFunction) as spy:
            LR.layer_reconstruction(qnn, layer, cali, batch_size=8, iters=iters, weight=0.01,
                                    asym=True, b_range=(20, 2), warmup=0.2, act_quant=False,
                                    opt_mode="mse")
        out[f"{tag}_w_perms"] = np.stack([p.numpy() for p in spy.perms]).astype(np.int64)
        out[f"{tag}_w_total_loss"] = np.array([r[1] for r in spy.rec], np.float64)
        out[f"{tag}_alpha"] = t2n(layer.weight_quantizer.alpha)
        with torch.no_grad():
            out[f"{tag}_what_hard"] = t2n(layer.weight_quantizer(layer.weight))
    qnn.set_quant_state(True, True)
    with torch.no_grad():
        qnn(cali[:8])
    qnn.disable_network_output_quantization()
    for tag, layer in layers:
        aq = layer.act_quantizer
        out[f"{tag}_a_delta0"] = np.array([float(aq.delta)], np.float32)
        out[f"{tag}_a_on"] = np.array([int(not aq.disable_act_quant and not layer.disable_act_quant)])
        torch.manual_seed(1005)
        with _Spy(LR.LossFunction) as spy:
            LR.layer_reconstruction(qnn, layer, cali, batch_size=8, iters=iters, act_quant=True,
                                    opt_mode="mse", lr=4e-4, p=2.4)
        out[f"{tag}_a_perms"] = np.stack([p.numpy() for p in spy.perms]).astype(np.int64)
        out[f"{tag}_a_total_loss"] = np.array([r[1] for r in spy.rec], np.float64)
        out[f"{tag}_a_delta"] = np.array([float(aq.delta)], np.float32)
    with torch.no_grad():
        out["logits"] = t2n(qnn(cali))
    out["iters"] = np.array([iters])
    save("recon_layer_brecq", **out)


FC_GRAD_STEPS = (0, 45, 199)


def gen_recon_layer_brecq_fc(iters=200, n_cali=64, bs=32, grad_steps=FC_GRAD_STEPS):
    """a22 on the fc loop as production runs it (the fused K19 pair, taken when C_in % 64 ==
    0): layer_reconstruction (quant/layer_recon.py:10-104, LossFunction :107-168) on the last
    layer of Linear(64, 512) -> ReLU -> Linear(512, 40) (40 = 2.5 16-row tiles: a
    partial tile as ResNet-18's 1000 outputs have), 8-bit by set_first_last_layer_to_8bit
    (quant_model.py:58-68) as ResNet-18's fc, asym capture (its input carries the first
    layer's 8-bit weights and the ReLU, as the fc's avgpool features do), batch 32 of 64
    cached samples, 200 iterations: the b schedule's warm-up (40 iterations), its decay and
    its end.  Recorded: the captured input / target, every batch draw, every iteration's
    rec (lp_loss) and total loss with the float64 rec loss at the fp32 run's own state (the
    reference's distance from exact arithmetic), V and its gradient before the Adam steps in
    grad_steps with the float64 gradient there, the final V and the hard W^."""
    import copy
    from quant import layer_recon as LR
    torch.manual_seed(1005)
    net = nn.Sequential(nn.Linear(64, 512), nn.ReLU(), nn.Linear(512, 40)).eval()
    wq = {"n_bits": 4, "channel_wise": True, "scale_method": "max", "tune_delta_zero": False,
          "symmetric": False}
    aq = {"n_bits": 8, "channel_wise": False, "scale_method": "max", "tune_delta_zero": False,
          "leaf_param": True, "symmetric": False}
    qnn = QuantModel(model=net, weight_quant_params=wq, act_quant_params=aq)
    qnn.eval()
    qnn.set_first_last_layer_to_8bit()
    torch.manual_seed(1005)
    cali = torch.randn(n_cali, 64)
    qnn.set_quant_state(True, False)
    with torch.no_grad():
        qnn(cali[:8])
    layer = qnn.model[2]
    assert isinstance(layer, QuantModule) and layer.weight_quantizer.n_bits == 8
    out = {"cali": t2n(cali)}
    _dump_qms(out, qnn, "")
    cache, recs, busy = {}, [], [False]
    orig_save, orig_lp = LR.save_inp_oup_data, LR.lp_loss

    def save_io(*a, **k):
        r = orig_save(*a, **k)
        cache["inp"], cache["out"] = r[0].clone(), r[1].clone()
        return r

    def lp(pred, tgt, p=2.0, reduction="none"):
        r = orig_lp(pred, tgt, p=p, reduction=reduction)
        if not busy[0]:
            busy[0] = True
            try:      # the same loss in float64 at this iteration's state and batch
                l64 = _to64(copy.deepcopy(layer))
                perm = spy.perms[-1][:bs]
                with torch.no_grad():
                    r64 = orig_lp(l64(cache["inp"][perm].double()), cache["out"][perm].double(),
                                  p=p, reduction=reduction)
                recs.append((float(r.item()), float(r64.item())))
            finally:
                busy[0] = False
        return r

    def truth(step):
        busy[0] = True
        try:
            l64 = _to64(copy.deepcopy(layer))
            q = l64.weight_quantizer
            q.alpha.grad = None
            lf = LR.LossFunction(l64, round_loss="relaxation", weight=0.01, max_count=iters,
                                 rec_loss="mse", b_range=(20, 2), decay_start=0, warmup=0.2, p=2.0)
            lf.count = step
            perm = spy.perms[-1][:bs]
            spy.orig_call(lf, l64(cache["inp"][perm].double()),
                          cache["out"][perm].double()).backward()
            return [np.asarray(q.alpha.grad.detach().numpy(), np.float64).copy()]
        finally:
            busy[0] = False

    LR.save_inp_oup_data, LR.lp_loss = save_io, lp
    try:
        torch.manual_seed(1005)
        with _Spy(LR.LossFunction) as spy, _GradSpy(grad_steps, truth) as gspy:
            LR.layer_reconstruction(qnn, layer, cali, batch_size=bs, iters=iters, weight=0.01,
                                    asym=True, b_range=(20, 2), warmup=0.2, act_quant=False,
                                    opt_mode="mse")
    finally:
        LR.save_inp_oup_data, LR.lp_loss = orig_save, orig_lp
    out["cached_inp"], out["cached_out"] = t2n(cache["inp"]), t2n(cache["out"])
    # the draws of N = 64: the batch is each draw's first bs entries
    out["perms"] = np.stack([p.numpy()[:bs] for p in spy.perms]).astype(np.int16)
    out["total_loss"] = np.array([r[1] for r in spy.rec], np.float64)
    out["rec_loss"] = np.array([r[0] for r in recs], np.float64)
    out["rec_loss64"] = np.array([r[1] for r in recs], np.float64)
    for s, (ps, gs) in sorted(gspy.rec.items()):
        out[f"gs{s}_V"], out[f"gs{s}_g"] = ps[0], gs[0]
        # the float64 gradient as its offset from the reference's fp32 one (fp32 holds the
        # offset to ~1e-7 of itself: far below either side's distance from it)
        out[f"gs{s}_t_minus_g"] = f32(gspy.rec64[s][0] - gs[0].astype(np.float64))
    out["grad_steps"] = np.array(sorted(gspy.rec), np.int64)
    q = layer.weight_quantizer
    out["V"] = t2n(q.alpha)
    with torch.no_grad():
        what = t2n(q(layer.weight))
    # the hard W^ as its 8-bit codes: (code - zp) * delta in fp32 gives it back bit for bit
    d, z = out["qm1_delta"][:, None], out["qm1_zp"][:, None]
    codes = np.rint(what / d + z)
    assert codes.min() >= 0 and codes.max() <= 255
    assert np.array_equal(((codes.astype(np.float32) - z) * d).view(np.int32), what.view(np.int32))
    out["what_hard_codes"] = codes.astype(np.uint8)
    out["iters"], out["bs"] = np.array([iters]), np.array([bs])
    save("recon_layer_brecq_fc", **out)


# ------------------------------------------------------------------ other block types
# ResNet-50 Bottleneck (config 3), MobileNetV2 InvertedResidual with a depthwise conv
# (config 4) and RegNetX ResBottleneckBlock with a grouped conv (config 5), each as the
# only block of a tiny net.  The reference's QuantModel needs setPathName on these block
# types (it is only defined on QuantBasicBlock): oracle-side shim below.
def _tiny_block_net(kind):
    torch.manual_seed(1005)
    if kind == "bottleneck":
        from models.resnet import Bottleneck
        ds = nn.Sequential(nn.Conv2d(16, 32, 1, stride=2, bias=False), nn.BatchNorm2d(32))
        blk, cout = Bottleneck(16, 8, stride=2, downsample=ds, norm_layer=nn.BatchNorm2d), 32
    elif kind == "inverted":
        from models.mobilenetv2 import InvertedResidual
        blk, cout = InvertedResidual(16, 16, 1, 2), 16
    else:
        from models.regnet import ResBottleneckBlock
        blk, cout = ResBottleneckBlock(16, 32, 2, 1.0, 8), 32
    net = nn.Sequential(nn.Conv2d(3, 16, 3, padding=1, bias=False), nn.BatchNorm2d(16), nn.ReLU(),
                        blk, nn.AdaptiveAvgPool2d(1), nn.Flatten(), nn.Linear(cout, 10))
    g = torch.Generator().manual_seed(7)
    for m in net.modules():
        if isinstance(m, nn.Conv2d):
            nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
        if isinstance(m, nn.BatchNorm2d):
            m.running_mean.copy_(torch.randn(m.num_features, generator=g) * 0.1)
            m.running_var.copy_(torch.rand(m.num_features, generator=g) + 0.5)
            m.weight.data.copy_(torch.rand(m.num_features, generator=g) + 0.5)
            m.bias.data.copy_(torch.randn(m.num_features, generator=g) * 0.1)
    return net.eval()


def _block_qnn(kind):
    from quant.quant_block import BaseQuantBlock
    if not hasattr(BaseQuantBlock, "setPathName"):
        BaseQuantBlock.setPathName = lambda self, n: setattr(self, "pathName", n)
    wq = {"n_bits": 2, "channel_wise": True, "scale_method": "max", "tune_delta_zero": False,
          "symmetric": False}
    aq = {"n_bits": 4, "channel_wise": False, "scale_method": "mse", "tune_delta_zero": False,
          "leaf_param": True, "symmetric": False}
    qnn = QuantModel(model=_tiny_block_net(kind), weight_quant_params=wq, act_quant_params=aq)
    qnn.eval()
    qnn.set_first_last_layer_to_8bit()
    return qnn


def _named_qms(block):
    return [(n, m) for n, m in block.named_modules() if isinstance(m, QuantModule)]


def gen_recon_blocks(iters=30, brecq_iters=10, n_cali=16, res=16):
    from quant.channelQuant import ChannelQuant
    for kind in ("bottleneck", "inverted", "resbottleneck"):
        out = {}
        # fused shifted-scale reconstruction
        qnn = _block_qnn(kind)
        torch.manual_seed(1005)
        cali = torch.randn(n_cali, 3, res, res)
        qnn.set_quant_state(True, False)
        with torch.no_grad():
            qnn(cali[:8])
        block = qnn.model[3]
        shift = [31 / 32, 33 / 32, 1.0]
        for n, m in _named_qms(block):
            out[f"f_{n}_w"], out[f"f_{n}_b"] = t2n(m.org_weight), t2n(m.org_bias)
            out[f"f_{n}_delta"] = t2n(m.weight_quantizer.delta.reshape(-1))
            out[f"f_{n}_zp"] = t2n(m.weight_quantizer.zero_point.reshape(-1))
            m.weight_quantizer = ChannelQuant(1.0, uaq=m.weight_quantizer, weight_tensor=m.org_weight.data,
                                              shiftTarget=shift, name="." + n)
            m.use_weight_quant = True
            m.cache_features = "none"
        qnn.set_quant_state(False, False)
        # the reference caches features only inside QuantBasicBlock.forward: capture this
        # block's FP input / output with a hook instead (same batches, same FP state)
        ins, outs = [], []
        def grab(mod, i, o):
            ins.append(i[0].detach().clone())
            outs.append(o.detach().clone())
        h = block.register_forward_hook(grab)
        with torch.no_grad():
            for i in range(n_cali // 8):
                qnn(cali[i * 8:(i + 1) * 8])
        h.remove()
        block.cached_inp_features, block.cached_out_features = [torch.cat(ins)], [torch.cat(outs)]
        MSM.set_quant_state_block(qnn, [BLOCK], "", True)
        out["f_cached_inp"] = t2n(torch.cat(block.cached_inp_features))
        out["f_cached_out"] = t2n(torch.cat(block.cached_out_features))
        torch.manual_seed(1005)
        with _Spy(LRF.FusedScaleLossFunction) as spy:
            res_loss = LRF.block_recon_fused_shiftedScale(block, iters, (0.01, 0.1), qnn, None)
        out["f_perms"] = np.stack([p.numpy() for p in spy.perms]).astype(np.int64)
        out["f_rec_loss"] = np.array([r[0] for r in spy.rec], np.float64)
        out["f_final_losses"] = np.array(res_loss, np.float64)
        for n, m in _named_qms(block):
            out[f"f_{n}_alpha"] = t2n(m.weight_quantizer.alpha)
            with torch.no_grad():
                out[f"f_{n}_what_hard"] = t2n(m.weight_quantizer(m.weight))
        # BRECQ AdaRound weight phase
        qnn = _block_qnn(kind)
        torch.manual_seed(1005)
        cali = torch.randn(n_cali, 3, res, res)
        qnn.set_quant_state(True, False)
        with torch.no_grad():
            qnn(cali[:8])
        block = qnn.model[3]
        out["b_cali"] = t2n(cali)
        qms = [m for m in qnn.modules() if isinstance(m, QuantModule)]
        for k, m in enumerate(qms):
            out[f"b_qm{k}_w"], out[f"b_qm{k}_b"] = t2n(m.org_weight), t2n(m.org_bias)
            out[f"b_qm{k}_delta"] = t2n(m.weight_quantizer.delta.reshape(-1))
            out[f"b_qm{k}_zp"] = t2n(m.weight_quantizer.zero_point.reshape(-1))
        torch.manual_seed(1005)
        with _Spy(BR.LossFunction) as spy:
            BR.block_reconstruction(qnn, block, cali, batch_size=8, iters=brecq_iters, weight=0.01,
                                    asym=True, b_range=(20, 2), warmup=0.2, act_quant=False,
                                    opt_mode="mse")
        out["b_total_loss"] = np.array([r[1] for r in spy.rec], np.float64)
        for n, m in _named_qms(block):
            out[f"b_{n}_alpha"] = t2n(m.weight_quantizer.alpha)
            with torch.no_grad():
                out[f"b_{n}_what_hard"] = t2n(m.weight_quantizer(m.weight))
        out["iters"] = np.array([iters, brecq_iters])
        save(f"recon_block_{kind}", **out)


# ------------------------------------------------------------------ round-2 goldens
def gen_act_quant():
    """ChannelQuantAct 'none' mode (channelQuantAct.py:36-67): per-tensor A4 q/dq at
    delta*shiftedScale with a [0, n-1] clamp and torch.round (no STE: d/dx = 0).  The
    delta/zero_point come from a UAQ 'mse' init on ReLU'd data; the evaluated tensor keeps
    negatives and large values so both clamp edges are hit."""
    from quant.channelQuantAct import ChannelQuantAct
    g = torch.Generator().manual_seed(1005)
    out = {}
    base = edge_tensor(g, (4, 6, 7, 7), 1.0)
    uaq = UniformAffineQuantizer(n_bits=4, channel_wise=False, scale_method="mse", leaf_param=True)
    with torch.no_grad():
        uaq(torch.relu(base))
    x = base * 1.5
    out["x"] = t2n(x)
    out["delta"] = t2n(uaq.delta.reshape(-1))
    out["zp"] = t2n(uaq.zero_point.reshape(-1))
    scales = (1.0, 33 / 32, 31 / 32, 0.5)
    out["scales"] = np.array(scales, np.float64)
    for k, s in enumerate(scales):
        q = ChannelQuantAct(uaq=uaq, shiftTarget=[1.0, 0.5])
        q.shiftedScale = s
        xr = x.clone().requires_grad_(True)
        y = q(xr)
        gy = torch.randn(x.shape, generator=g)
        uaq.delta.grad = None
        uaq.zero_point.grad = None
        (y * gy).sum().backward()
        out[f"s{k}_y"] = t2n(y)
        out[f"s{k}_gy"] = t2n(gy)
        out[f"s{k}_gx"] = t2n(xr.grad) if xr.grad is not None else np.zeros(x.shape, np.float32)
        out[f"s{k}_gdelta"] = t2n(uaq.delta.grad.reshape(-1))
        out[f"s{k}_gzp"] = t2n(uaq.zero_point.grad.reshape(-1))
    save("act_quant", **out)


def gen_recon_layer_fused(iters=30, n_cali=16, res=16):
    """a19: layer_recon_fused_shiftedScale raises UnboundLocalError in the reference
    (`opt_params += ...` before assignment, layer_recon_fused_shiftedScale.py:156).  Its
    evident intent -- the fused loop on ONE QuantModule with p = 1 (:165) and Adam's
    default lr (= the block loop's 1e-3) -- is run here by the reference's own block loop
    (block_recon_fused_shiftedScale accepts a QuantModule: named_modules() yields it) with
    the loss class pinned to p = 1.  The layer variant's post-loop flags (:207-211: hard
    targets + shiftedDone, hard_round only on the LAYER when adaround) are then applied
    and the 'Hard Round' loss evaluated the way :212-215 do."""
    qnn = _build_tiny_qnn()
    torch.manual_seed(1005)
    cali = torch.randn(n_cali, 3, res, res)
    qnn.set_quant_state(True, False)
    with torch.no_grad():
        qnn(cali[:8])
    shift = [31 / 32, 33 / 32, 1.0]
    MSM.build_ShiftedChannelQuant(qnn, [BLOCK], "", shiftTarget=shift, skipShiftLayer=[])
    qnn.set_quant_state(False, False)
    layer = BLOCK + ".conv1"
    _cache(qnn, [layer], cali, 8)
    m = qnn.model[3].conv1
    m.use_weight_quant = True
    q = m.weight_quantizer
    out = {"w": t2n(m.org_weight), "b": t2n(m.org_bias), "delta": t2n(q.delta.reshape(-1)),
           "zp": t2n(q.zero_point.reshape(-1)),
           "cached_inp": t2n(torch.cat(m.cached_inp_features)),
           "cached_out": t2n(torch.cat(m.cached_out_features))}
    orig = LRF.FusedScaleLossFunction

    class _P1(orig):
        def __init__(self, *a, **k):
            k["p"] = 1.0
            super().__init__(*a, **k)

    LRF.FusedScaleLossFunction = _P1
    try:
        torch.manual_seed(1005)
        with _Spy(_P1) as spy:
            res_loss = LRF.block_recon_fused_shiftedScale(m, iters, (0.01, 0.1), qnn, None)
    finally:
        LRF.FusedScaleLossFunction = orig
    out["perms"] = np.stack([p.numpy() for p in spy.perms]).astype(np.int64)
    out["rec_loss"] = np.array([r[0] for r in spy.rec], np.float64)
    out["total_loss"] = np.array([r[1] for r in spy.rec], np.float64)
    out["soft_loss"] = np.array([res_loss[0]], np.float64)
    out["alpha"] = t2n(q.alpha)
    out["beta0"] = t2n(q.beta)
    # the layer variant's flags: hard targets, SOFT rounding (hard_round untouched, :207-211)
    q.hard_round = False
    q.hard_targets = True
    q.shiftedDone = True
    inp = torch.cat(m.cached_inp_features)[:32]
    tgt = torch.cat(m.cached_out_features)[:32]
    with torch.no_grad():
        out["hard_loss"] = np.array([float(lp_loss(m(inp), tgt, p=1.0))], np.float64)
        out["what_layer_hard"] = t2n(q(m.weight))
        q.hard_round = True
        out["what_hard"] = t2n(q(m.weight))
    out["iters"] = np.array([iters])
    save("recon_layer_fused", **out)


def gen_recon_block_shift(iters=20, n_cali=16, res=16):
    """a21: block_recon_shiftedScale (layer_recon_shiftedScale.py:12-124 +
    ScaleLossBlockFunction :340-412), shift phase (init_v, learned_hard_sigmoid, entropy
    regulariser) then adaround phase (update_delta, init_beta, beta) on the tiny net's
    BasicBlock at W2."""
    qnn = _build_tiny_qnn()
    torch.manual_seed(1005)
    cali = torch.randn(n_cali, 3, res, res)
    qnn.set_quant_state(True, False)
    with torch.no_grad():
        qnn(cali[:8])
    shift = [31 / 32, 33 / 32, 1.0]
    MSM.build_ShiftedChannelQuant(qnn, [BLOCK], "", shiftTarget=shift, skipShiftLayer=[])
    qnn.set_quant_state(False, False)
    _cache(qnn, [BLOCK], cali, 8)
    MSM.set_quant_state_block(qnn, [BLOCK], "", True)
    block = qnn.model[3]
    out = {}
    _dump_block(out, block)
    for n in CONVS:
        q = getattr(block, n).weight_quantizer
        out[n + "_delta"] = t2n(q.delta.reshape(-1))
        out[n + "_zp"] = t2n(q.zero_point.reshape(-1))
    out["cached_inp"] = t2n(torch.cat(block.cached_inp_features))
    out["cached_out"] = t2n(torch.cat(block.cached_out_features))
    torch.manual_seed(1005)
    with _Spy(LRS.ScaleLossBlockFunction) as spy:
        l1 = LRS.block_recon_shiftedScale(block, iters, 0.1, qnn, None)
    out["s_perms"] = np.stack([p.numpy() for p in spy.perms]).astype(np.int64)
    out["s_rec_loss"] = np.array([r[0] for r in spy.rec], np.float64)
    out["s_total_loss"] = np.array([r[1] for r in spy.rec], np.float64)
    out["s_final"] = np.array(l1, np.float64)
    for n in CONVS:
        m = getattr(block, n)
        q = m.weight_quantizer
        out[n + "_s_alpha"] = t2n(q.alpha)
        with torch.no_grad():
            out[n + "_s_what"] = t2n(q(m.weight))       # hard targets (lhs mode)
    with _Spy(LRS.ScaleLossBlockFunction) as spy:
        l2 = LRS.block_recon_shiftedScale(block, iters, 0.01, qnn, None, adaround=True)
    out["a_perms"] = np.stack([p.numpy() for p in spy.perms]).astype(np.int64)
    out["a_rec_loss"] = np.array([r[0] for r in spy.rec], np.float64)
    out["a_total_loss"] = np.array([r[1] for r in spy.rec], np.float64)
    out["a_final"] = np.array(l2, np.float64)
    for n in CONVS:
        m = getattr(block, n)
        q = m.weight_quantizer
        out[n + "_a_delta"] = t2n(q.delta)
        out[n + "_a_beta"] = t2n(q.beta)
        with torch.no_grad():
            out[n + "_a_what"] = t2n(q(m.weight))       # hard rounding (adaround mode)
    out["iters"] = np.array([iters])
    save("recon_block_shift", **out)


def _tiny_net2():
    """stem -> BasicBlock(16->16) -> BasicBlock(16->32, stride 2, downsample) -> pool -> fc:
    two reconstructable blocks, so the second block's cached input carries the first
    block's finished (hard) quantization, as in the driver (ShiftedScaleQuant.py:236-256)."""
    from models.resnet import BasicBlock
    torch.manual_seed(1005)
    ds = nn.Sequential(nn.Conv2d(16, 32, 1, stride=2, bias=False), nn.BatchNorm2d(32))
    net = nn.Sequential(nn.Conv2d(3, 16, 3, padding=1, bias=False), nn.BatchNorm2d(16), nn.ReLU(),
                        BasicBlock(16, 16, norm_layer=nn.BatchNorm2d),
                        BasicBlock(16, 32, stride=2, downsample=ds, norm_layer=nn.BatchNorm2d),
                        nn.AdaptiveAvgPool2d(1), nn.Flatten(), nn.Linear(32, 10))
    g = torch.Generator().manual_seed(7)
    for m in net.modules():
        if isinstance(m, nn.Conv2d):
            nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
        if isinstance(m, nn.BatchNorm2d):
            m.running_mean.copy_(torch.randn(m.num_features, generator=g) * 0.1)
            m.running_var.copy_(torch.rand(m.num_features, generator=g) + 0.5)
            m.weight.data.copy_(torch.rand(m.num_features, generator=g) + 0.5)
            m.bias.data.copy_(torch.randn(m.num_features, generator=g) * 0.1)
    return net.eval()


def _build_tiny_qnn2(bits_w=2, bits_a=4):
    wq = {"n_bits": bits_w, "channel_wise": True, "scale_method": "max", "tune_delta_zero": False,
          "symmetric": False}
    aq = {"n_bits": bits_a, "channel_wise": False, "scale_method": "mse", "tune_delta_zero": False,
          "leaf_param": True, "symmetric": False}
    qnn = QuantModel(model=_tiny_net2(), weight_quant_params=wq, act_quant_params=aq)
    qnn.eval()
    qnn.set_first_last_layer_to_8bit()
    return qnn


def _dump_qms(out, qnn, prefix):
    qms = [m for m in qnn.modules() if isinstance(m, QuantModule)]
    for k, m in enumerate(qms):
        out[f"{prefix}qm{k}_w"], out[f"{prefix}qm{k}_b"] = t2n(m.org_weight), t2n(m.org_bias)
        out[f"{prefix}qm{k}_delta"] = t2n(m.weight_quantizer.delta.reshape(-1))
        out[f"{prefix}qm{k}_zp"] = t2n(m.weight_quantizer.zero_point.reshape(-1))
        out[f"{prefix}qm{k}_bits"] = np.array([m.weight_quantizer.n_bits])


def gen_driver(iters=20, n_cali=16, res=16):
    """a23 + (f1): the shipped fused driver flow (channelShift_wLoss,
    ShiftedScaleQuant.py:185-286) over BOTH blocks of a two-block net, with the
    reference's own helpers: build_ShiftedChannelQuant, per block the 'if' cache under the
    current quant state (earlier blocks finished and weight-quantized) and the FP 'of'
    cache, set_quant_state_block, QuantRecursiveShiftRecon -> run_ShiftReconFused ->
    block_recon_fused_shiftedScale, clear_cached_features; then the weight-quantized
    network's logits.  Every block's cached features are recorded (the feature-cache
    parity of SURVEY §8(f) row 1)."""
    ssq_mod = types.ModuleType("data.cifar10")
    ssq_mod.build_cifar10_data = lambda *a, **k: (None, None)
    img_mod = types.ModuleType("data.imagenet")
    img_mod.build_imagenet_data = lambda *a, **k: (None, None)
    sys.modules.setdefault("data", types.ModuleType("data"))
    sys.modules["data.cifar10"], sys.modules["data.imagenet"] = ssq_mod, img_mod
    import ShiftedScaleQuant as SSQD
    qnn = _build_tiny_qnn2()
    torch.manual_seed(1005)
    cali = torch.randn(n_cali, 3, res, res)
    qnn.set_quant_state(True, False)
    with torch.no_grad():
        qnn(cali[:8])
    out = {"cali": t2n(cali)}
    _dump_qms(out, qnn, "")
    shift = [31 / 32, 33 / 32, 1.0]
    layers = [".model.3", ".model.4"]
    MSM.build_ShiftedChannelQuant(qnn, layers, "", shiftTarget=shift, skipShiftLayer=[])
    qnn.set_quant_state(False, False)
    loss_dic = {}
    torch.manual_seed(1005)
    for k, layer in enumerate(layers):
        _cache(qnn, [layer], cali, 8)
        block = qnn.model[3 + k]
        out[f"b{k}_cached_inp"] = t2n(torch.cat(block.cached_inp_features))
        out[f"b{k}_cached_out"] = t2n(torch.cat(block.cached_out_features))
        MSM.set_quant_state_block(qnn, [layer], "", True)
        with _Spy(LRF.FusedScaleLossFunction) as spy, \
                _GradSpy((0, 5, iters - 1), _fused_truth(block, spy, (0.01, 0.1), iters)) as gspy:
            SSQD.QuantRecursiveShiftRecon(qnn, [layer], qnn, None, "", loss_dic, iters=iters,
                                          lmda=0.1, shiftTarget=shift)
        gspy.dump(out, f"b{k}_")
        qnn.clear_cached_features()
        out[f"b{k}_losses"] = np.array(loss_dic[layer][0], np.float64)
        names = ("conv1", "conv2") + (("downsample",) if k == 1 else ())
        for n in names:
            m = getattr(block, n)
            q = m.weight_quantizer
            out[f"b{k}_{n}_alpha"] = t2n(q.alpha)
            out[f"b{k}_{n}_beta0"] = t2n(q.beta)
            with torch.no_grad():
                out[f"b{k}_{n}_what_hard"] = t2n(q(m.weight))
    qnn.set_quant_state(True, False)
    with torch.no_grad():
        out["logits"] = t2n(qnn(cali))
    out["iters"] = np.array([iters])
    save("recon_driver", **out)


def gen_wmse_driver(n_cali=16, res=16):
    """a23: the shipped default path `ShiftedScaleQuant.py --test=True` ->
    channelShift_wMSE (:119-183): UAQ weight init on cali[:64], then every QuantModule not
    in layerDisabled (only the fc there) and not ignore_reconstruction gets a
    ChannelQuantMSE(opt_mode='max', level, threshold) through the reference's own
    build_ShiftedChannelQuantMSELayer, whose init_scale picks the input scales.  The walk
    is channelShift_wMSE's nested build_ShiftedChannelQuantMSE, restated here (it is a
    closure the reference does not export).  Recorded: each layer's inp_scale and the
    weight-quantized network's logits (validate_with_loss's forward)."""
    out = {}
    for level, thr in ((1, 1.0), (8, 2.0), (64, 2.0)):
        qnn = _build_tiny_qnn2()
        torch.manual_seed(1005)
        cali = torch.randn(n_cali, 3, res, res)
        qnn.set_quant_state(True, False)
        with torch.no_grad():
            qnn(cali[:8])
        tag = f"l{level}"
        if level == 1:
            out["cali"] = t2n(cali)
            _dump_qms(out, qnn, "")
        layer_disabled = [".model.7"]
        kw = dict(shiftTarget=[31 / 32, 33 / 32, 1.0], level=level, threshold=thr, opt_mode="max")
        built = []

        def walk(model, prv_name=""):
            from quant.quant_block import QuantBasicBlock
            for name, module in model.named_children():
                cur = prv_name + "." + name
                if isinstance(module, QuantModule):
                    if module.ignore_reconstruction is True:
                        continue
                    if cur not in layer_disabled:
                        MSM.build_ShiftedChannelQuantMSELayer(model, cur, module, 1.0, **kw)
                        built.append(cur)
                elif isinstance(module, QuantBasicBlock):
                    if module.ignore_reconstruction is True:
                        continue
                    if cur in layer_disabled:
                        MSM.build_ShiftedChannelQuantMSEBlock(model, cur, module, 1.0, **kw)
                    else:
                        walk(module, cur)
                else:
                    walk(module, cur)

        walk(qnn)
        out[f"{tag}_names"] = np.array(built)
        qms = [m for m in qnn.modules() if isinstance(m, QuantModule)]
        for k, m in enumerate(qms):
            if isinstance(m.weight_quantizer, ChannelQuantMSE):
                out[f"{tag}_qm{k}_inp_scale"] = t2n(m.weight_quantizer.inp_scale)
                with torch.no_grad():
                    out[f"{tag}_qm{k}_what"] = t2n(m.weight_quantizer(m.org_weight))
        with torch.no_grad():
            out[f"{tag}_logits"] = t2n(qnn(cali))
        out[f"{tag}_thr"] = np.array([thr])
    save("driver_wmse", **out)


def gen_validate(n_cali=16, n_val=40, res=16, bs=8):
    """(f3) W2A4 fake-quant validation inference: weights UAQ 'max' (8-bit stem/head), acts
    UAQ 'mse' initialised by one forward over cali[:8] under set_quant_state(True, True),
    network output left unquantized (disable_network_output_quantization), then the
    reference's own common.validate_model over a labelled synthetic set.  Half of the labels
    are the FP network's predictions so top-1 is not chance.  Recorded: every act
    quantizer's delta / zero_point, the quantized logits and the reference's top-1."""
    import common as C
    qnn = _build_tiny_qnn2()
    torch.manual_seed(1005)
    cali = torch.randn(n_cali, 3, res, res)
    val = torch.randn(n_val, 3, res, res)
    out = {"cali": t2n(cali), "val": t2n(val)}
    with torch.no_grad():
        fp = qnn(val)
    g = torch.Generator().manual_seed(11)
    labels = torch.randint(0, 10, (n_val,), generator=g)
    labels[: n_val // 2] = fp[: n_val // 2].argmax(1)
    qnn.set_quant_state(True, True)
    with torch.no_grad():
        qnn(cali[:8])
    qnn.disable_network_output_quantization()
    _dump_qms(out, qnn, "")
    # every act quantizer (QuantModules and the blocks' output quantizers), in module order
    owners = [m for m in qnn.modules() if hasattr(m, "act_quantizer")]
    for k, m in enumerate(owners):
        aq = m.act_quantizer
        out[f"aq{k}_kind"] = np.array([type(m).__name__])
        out[f"aq{k}_bits"] = np.array([aq.n_bits])
        out[f"aq{k}_on"] = np.array([int(m.use_act_quant and not getattr(m, "disable_act_quant", False))])
        if aq.delta is not None and aq.inited:
            out[f"aq{k}_delta"] = t2n(torch.as_tensor(aq.delta).reshape(-1))
            out[f"aq{k}_zp"] = t2n(torch.as_tensor(aq.zero_point).reshape(-1))
    loader = [(val[i:i + bs], labels[i:i + bs]) for i in range(0, n_val, bs)]
    top1 = C.validate_model(loader, qnn)
    with torch.no_grad():
        out["logits"] = t2n(qnn(val))
    out["labels"] = labels.numpy().astype(np.int64)
    out["top1"] = np.array([float(top1)], np.float64)
    out["bs"] = np.array([bs])
    save("validate_w2a4", **out)


# ------------------------------------------------------------------ round-3: real shapes
def _real_block(kind, cin, cout):
    """The reference's own block classes at the real channel counts (realshape.CASES)."""
    if kind == "basic1":
        from models.resnet import BasicBlock
        return BasicBlock(cin, cout, norm_layer=nn.BatchNorm2d)
    if kind == "basic":
        from models.resnet import BasicBlock
        ds = nn.Sequential(nn.Conv2d(cin, cout, 1, stride=2, bias=False), nn.BatchNorm2d(cout))
        return BasicBlock(cin, cout, stride=2, downsample=ds, norm_layer=nn.BatchNorm2d)
    if kind == "bottleneck":
        from models.resnet import Bottleneck
        ds = nn.Sequential(nn.Conv2d(cin, cout, 1, stride=1, bias=False), nn.BatchNorm2d(cout))
        return Bottleneck(cin, cout // 4, stride=1, downsample=ds, norm_layer=nn.BatchNorm2d)
    if kind == "inverted":
        from models.mobilenetv2 import InvertedResidual
        return InvertedResidual(cin, cout, 1, 6)
    from models.regnet import ResBottleneckBlock
    return ResBottleneckBlock(cin, cout, 2, 1.0, 48)


def _real_qnn(case, bits_w=2, bits_a=4):
    from quant.quant_block import BaseQuantBlock
    import realshape as RS
    if not hasattr(BaseQuantBlock, "setPathName"):
        BaseQuantBlock.setPathName = lambda self, n: setattr(self, "pathName", n)
    kind, cin, cout, _ = RS.CASES[case]
    net = RS.seed_net(RS.wrap(_real_block(kind, cin, cout), cout))
    lay = (RS.layout(net), RS.seed_sha(net))
    wq = {"n_bits": bits_w, "channel_wise": True, "scale_method": "max", "tune_delta_zero": False,
          "symmetric": False}
    aq = {"n_bits": bits_a, "channel_wise": False, "scale_method": "mse", "tune_delta_zero": False,
          "leaf_param": True, "symmetric": False}
    qnn = QuantModel(model=net, weight_quant_params=wq, act_quant_params=aq)
    qnn.eval()
    return qnn, lay


def _dump_sub(out, key, a, idx):
    a = np.asarray(a, np.float32).reshape(-1)
    out[key + "_sub"] = a[idx]
    out[key + "_max"] = np.array([np.abs(a).max(initial=0.0)], np.float64)


def _real_fused(case, x, iters, grad_steps, bias_cal, out, keep_cached=True):
    """The fused shifted-scale loop (block_recon_fused_shiftedScale) on the real-shape case:
    the recorded inputs (weight hashes, deltas / zero points, the FP block output), the
    batch draws, per-iteration losses, values / gradients (+ the float64 truth) at
    grad_steps, final alpha (and gamma^z / phi^z with bias_cal) and hard-weight hashes."""
    import contextlib
    import realshape as RS
    from quant.channelQuant import ChannelQuant
    shift = [31 / 32, 33 / 32, 1.0]
    qnn, _ = _real_qnn(case)
    block = qnn.model[0]
    qnn.set_quant_state(True, False)
    with torch.no_grad():
        qnn(x)
    qms = _named_qms(block)
    out["qms"] = np.array([n for n, _ in qms])
    for n, m in qms:
        out[f"{n}_w_sha"] = np.array([RS.sha(t2n(m.org_weight))])
        out[f"{n}_b_sha"] = np.array([RS.sha(t2n(m.org_bias))])
        out[f"{n}_delta"] = t2n(m.weight_quantizer.delta.reshape(-1))
        out[f"{n}_zp"] = t2n(m.weight_quantizer.zero_point.reshape(-1))
        m.weight_quantizer = ChannelQuant(1.0, uaq=m.weight_quantizer, weight_tensor=m.org_weight.data,
                                          shiftTarget=shift, name="." + n)
        m.use_weight_quant = True
        m.cache_features = "none"
    qnn.set_quant_state(False, False)
    with torch.no_grad():
        fp = block(x)
    if keep_cached:
        out["cached_out"] = t2n(fp)
    out["cached_out_sha"] = np.array([RS.sha(t2n(fp))])
    block.cached_inp_features, block.cached_out_features = [x.clone()], [fp.clone()]
    MSM.set_quant_state_block(qnn, [".model.0"], "", True)
    for n, m in qms:
        out[f"{n}_beta0_sha"] = np.array([RS.sha(t2n(m.weight_quantizer.beta))]) \
            if getattr(m.weight_quantizer, "beta", None) is not None else np.array([""])
    torch.manual_seed(1005)
    with _Spy(LRF.FusedScaleLossFunction) as spy, \
            (_BiasCalAdam(block) if bias_cal else contextlib.nullcontext()):
        with _GradSpy(grad_steps, _fused_truth(block, spy, (0.01, 0.1), iters, bias_cal=bias_cal)) as gspy:
            res_loss = LRF.block_recon_fused_shiftedScale(block, iters, (0.01, 0.1), qnn, None)
    out["perms"] = np.stack([p.numpy() for p in spy.perms]).astype(np.int64)
    out["rec_loss"] = np.array([r[0] for r in spy.rec], np.float64)
    out["final_losses"] = np.array(res_loss, np.float64)
    out["iters"] = np.array([iters])
    gspy.dump(out)      # alpha is [C_in, S], gamma / phi [1, C_out, 1, 1]: small, kept whole
    for j, (n, m) in enumerate(qms):
        q = m.weight_quantizer
        out[f"{n}_alpha"] = t2n(q.alpha)
        out[f"{n}_gamma"] = t2n(m.alpha_out)
        out[f"{n}_phi"] = t2n(m.beta_out)
        bt = t2n(q.beta)
        out[f"{n}_beta_sha"] = np.array([RS.sha(bt)])
        out[f"{n}_beta_sub"] = bt.reshape(-1)[RS.sub_idx(bt.size)]
        with torch.no_grad():
            out[f"{n}_what_hard_sha"] = np.array([RS.sha(t2n(q(m.weight)))])
    return qms


def gen_real_layer_shift(case="r18_layer1_0", iters=20):
    """Config 1 (W4A8, layer_recon_shiftedScale, layer_recon_shiftedScale.py:262-338 +
    ScaleLossFunction :414-486) at the real ResNet-18 layer1.0.conv1 shape (64 -> 64, 3x3):
    the shift phase (init_v, learned_hard_sigmoid, entropy regulariser, lambda 0.1) then the
    AdaRound phase (update_delta, init_beta, beta, lambda 0.01), as gen_recon_layer_shift
    does on the toy conv.  Recorded: the conv's cached FP output (the loop's target), batch
    draws, per-iteration losses, the shift logits with their values / gradients (+ float64
    truth) at the recorded steps, the selected per-(Co, Ci) delta, the final beta and the
    hashes of the hard weights of both phases."""
    import realshape as RS
    x = RS.calib_input(case)
    qnn, (lay, ssha) = _real_qnn(case, bits_w=4, bits_a=8)
    out = {"layout": np.array(lay), "seed_sha": np.array([ssha])}
    qnn.set_quant_state(True, False)
    with torch.no_grad():
        qnn(x)
    block_name, layer_name = ".model.0", ".model.0.conv1"
    MSM.build_ShiftedChannelQuant(qnn, [block_name], "", shiftTarget=[31 / 32, 33 / 32, 1.0],
                                  skipShiftLayer=[])
    qnn.set_quant_state(False, False)
    _cache(qnn, [layer_name], x, RS.N_CALI)
    m = qnn.model[0].conv1
    m.use_weight_quant = True
    q = m.weight_quantizer
    out["w_sha"] = np.array([RS.sha(t2n(m.org_weight))])
    out["b_sha"] = np.array([RS.sha(t2n(m.org_bias))])
    out["delta"] = t2n(q.delta.reshape(-1))
    out["zp"] = t2n(q.zero_point.reshape(-1))
    out["cached_out"] = t2n(torch.cat(m.cached_out_features))
    torch.manual_seed(1005)
    with _Spy(LRS.ScaleLossFunction) as spy, \
            _GradSpy((0, 5, iters - 1), _layer_truth(m, spy, 0.1, iters, False)) as gspy:
        l1 = LRS.layer_recon_shiftedScale(m, iters, 0.1, qnn, None)
    gspy.dump(out, "shift_")
    out["shift_perms"] = np.stack([p.numpy() for p in spy.perms]).astype(np.int64)
    out["shift_total_loss"] = np.array([r[1] for r in spy.rec], np.float64)
    out["shift_final"] = np.array(l1, np.float64)
    out["shift_alpha"] = t2n(q.alpha)
    out["shift_xq_sha"] = np.array([RS.sha(np.stack([t2n(t) for t in q.x_q]))])
    with torch.no_grad():
        out["shift_what_sha"] = np.array([RS.sha(t2n(q(m.weight)))])
    q.hard_targets = False
    # the AdaRound phase's beta gradients (ScaleLossFunction's lp term + the rounding term,
    # :297-338,414-486) at the same steps, with their float64 truth
    with _Spy(LRS.ScaleLossFunction) as spy, \
            _GradSpy((0, 5, iters - 1), _layer_truth(m, spy, 0.01, iters, True)) as gspy:
        l2 = LRS.layer_recon_shiftedScale(m, iters, 0.01, qnn, None, adaround=True)
    gspy.dump(out, "ar_")
    out["ar_perms"] = np.stack([p.numpy() for p in spy.perms]).astype(np.int64)
    out["ar_total_loss"] = np.array([r[1] for r in spy.rec], np.float64)
    out["ar_final"] = np.array(l2, np.float64)
    out["ar_delta"] = t2n(q.delta)
    out["ar_beta"] = t2n(q.beta)
    with torch.no_grad():
        out["ar_what_sha"] = np.array([RS.sha(t2n(q(m.weight)))])
    out["iters"] = np.array([iters])
    save(f"real_{case}_layer_shift_w4a8", **out)


def gen_real_biascal(cases=("r18_layer4_0", "r18_layer1_0")):
    """--bias_cal at the real shapes: the fused loop under _BiasCalAdam (alpha, gamma^z and
    phi^z learned), 20 iterations, values / gradients / float64 truth at GRAD_STEPS."""
    import realshape as RS
    for case in cases:
        out = {}
        _real_fused(case, RS.calib_input(case), RS.ITERS, RS.GRAD_STEPS, True, out, keep_cached=False)
        save(f"real_{case}_biascal", **out)


def gen_long_horizon(case="r18_layer1_0"):
    """The driver's horizon: 625 iterations of block_recon_fused_shiftedScale
    (ShiftedScaleQuant.py:53-55; the b / b2 schedules end at iters and 3/4 iters,
    layer_recon_fused_shiftedScale.py:246-250,382-399) on the ResNet-18 layer1.0 shape, as
    shipped and with --bias_cal.  The FP block output is the one in real_<case>.npz
    (checked by hash)."""
    import realshape as RS
    x = RS.calib_input(case)
    for bias_cal in (False, True):
        out = {}
        _real_fused(case, x, RS.LONG_ITERS, RS.LONG_GRAD_STEPS, bias_cal, out, keep_cached=False)
        save(f"long_{case}" + ("_biascal" if bias_cal else ""), **out)


def gen_real_shapes(cases=None):
    """Reference-pinned parity at the real block shapes of configs 2-5 (realshape.CASES):
    the fused shifted-scale loop (block_recon_fused_shiftedScale, 20 iterations) and BRECQ's
    AdaRound block reconstruction (10 iterations) on 8 calibration inputs.  Weights and
    inputs are regenerated from integer seeds on both sides; recorded are the reference's
    folded-weight hashes, weight quantizer deltas / zero points, FP block outputs,
    per-iteration losses and batch draws, the shift logits alpha ([C_in, S]) with their value
    and gradient at GRAD_STEPS, BRECQ's AdaRound V ([C_out, ...], full weight size:
    sub-sampled at fixed entries with its max-abs, per-output-channel gradient L1 norms and
    the packed sign bits that decide the hard rounding) and the hashes of the final hard
    weights."""
    import realshape as RS
    for case in (cases or RS.CASES):
        kind, cin, cout, _ = RS.CASES[case]
        x = RS.calib_input(case)
        lay, ssha = _real_qnn(case)[1]
        out = {"layout": np.array(lay), "seed_sha": np.array([ssha])}
        # ---- fused shifted-scale loop
        _real_fused(case, x, RS.ITERS, RS.GRAD_STEPS, False, out)
        # ---- BRECQ AdaRound block reconstruction
        qnn, _ = _real_qnn(case)
        block = qnn.model[0]
        qnn.set_quant_state(True, False)
        with torch.no_grad():
            qnn(x)
        qms = _named_qms(block)
        torch.manual_seed(1005)
        with _Spy(BR.LossFunction) as spy, _GradSpy(RS.BRECQ_GRAD_STEPS) as gspy:
            BR.block_reconstruction(qnn, block, x, batch_size=8, iters=RS.BRECQ_ITERS, weight=0.01,
                                    asym=True, b_range=(20, 2), warmup=0.2, act_quant=False,
                                    opt_mode="mse")
        out["b_perms"] = np.stack([p.numpy() for p in spy.perms]).astype(np.int64)
        out["b_total_loss"] = np.array([r[1] for r in spy.rec], np.float64)
        for j, (n, m) in enumerate(qms):
            q = m.weight_quantizer
            v = t2n(q.alpha)
            idx = RS.sub_idx(v.size)          # fixed entries: the test re-derives them
            _dump_sub(out, f"b_{n}_V", v, idx)
            out[f"b_{n}_V_pos"] = np.packbits((v >= 0).reshape(-1))
            for s_ in RS.BRECQ_GRAD_STEPS:
                g = gspy.rec[s_][1][j]
                _dump_sub(out, f"b_{n}_gs{s_}", g, idx)
                out[f"b_{n}_gs{s_}_rowl1"] = RS.row_l1(g)
            with torch.no_grad():
                out[f"b_{n}_what_hard_sha"] = np.array([RS.sha(t2n(q(m.weight)))])
        save(f"real_{case}", **out)


if __name__ == "__main__":
    which = sys.argv[1:] or ["uaq", "channelquant", "adaround", "specials", "inpscale", "loss", "recon",
                             "layershift", "brecq", "blocks", "act", "layerfused", "blockshift", "driver",
                             "wmse", "validate", "real", "recon_biascal", "real_biascal", "long",
                             "layerbrecq", "reallayer", "brecq_long", "brecq_affine", "init_specials",
                             "layerbrecq_fc"]
    torch.set_num_threads(4)
    if "uaq" in which:
        gen_uaq()
    if "channelquant" in which:
        gen_channelquant()
    if "adaround" in which:
        gen_adaround()
    if "specials" in which:
        gen_uaq_specials()
        gen_channelquant(specials=True)
        gen_adaround(specials=True)
    if "init_specials" in which:
        gen_init_specials()
    if "inpscale" in which:
        gen_inpscale()
    if "loss" in which:
        gen_loss()
    if "recon" in which:
        gen_recon_fused()
    if "layershift" in which:
        gen_recon_layer_shift()
    if "brecq" in which:
        gen_recon_brecq()
    if "brecq_long" in which:
        gen_recon_brecq(iters=400, name="recon_brecq_long")
    if "brecq_affine" in which:
        gen_recon_brecq(iters=50, name="recon_brecq_affine", affine=True)
    if "blocks" in which:
        gen_recon_blocks()
    if "act" in which:
        gen_act_quant()
    if "layerfused" in which:
        gen_recon_layer_fused()
    if "blockshift" in which:
        gen_recon_block_shift()
    if "driver" in which:
        gen_driver()
    if "wmse" in which:
        gen_wmse_driver()
    if "validate" in which:
        gen_validate()
    if "real" in which:
        gen_real_shapes()
    if "reallayer" in which:
        gen_real_layer_shift()
    if "layerbrecq" in which:
        gen_recon_layer_brecq()
    if "layerbrecq_fc" in which:
        gen_recon_layer_brecq_fc()
    if "recon_biascal" in which:
        gen_recon_fused(bias_cal=True)
    if "real_biascal" in which:
        gen_real_biascal()
    if "long" in which:
        gen_long_horizon()
