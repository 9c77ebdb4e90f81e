"""Tensor-level wrappers and autograd Functions over libssq.so.

Each function states the reference op sequence it replaces.  All of them require fp32
tensors on the HIP device; nothing here falls back to eager PyTorch arithmetic.
Weight geometry: W is (Co, Ci, kh, kw) -> (Co, Ci, K=kh*kw), Linear (Co, Ci) -> K = 1.
"""
import ctypes as C
import os

import torch

from . import _capi as A
from ._capi import call, fptr, query, stream_of, workspace


def qrange(n_bits, sym):
    n = 2 ** n_bits
    return (-(n // 2), n // 2 - 1) if sym else (0, n - 1)


def geometry(w):
    if w.dim() == 4:
        return int(w.shape[0]), int(w.shape[1]), int(w.shape[2] * w.shape[3]), 0
    if w.dim() == 2:
        return int(w.shape[0]), int(w.shape[1]), 1, 1
    raise ValueError(f"weight must be 2-D (Linear) or 4-D (Conv2d), got {tuple(w.shape)}")


def _codes_buf(x, want):
    return torch.empty(x.shape, dtype=torch.uint8, device=x.device) if want else None


def _vp(t):
    return None if t is None else C.c_void_p(t.data_ptr())


# ------------------------------------------------------------------ K1/K2
def _channel_layout(x, delta):
    """(inner, nch) for ssq_fq_fwd: delta broadcasts over x as x.shape[:k] + (1,)*rest,
    channel c of element i = (i // inner) % nch."""
    nd = delta.numel()
    if nd == 1:
        return 1, 1
    ds = tuple(delta.shape) + (1,) * (x.dim() - delta.dim())
    for k in range(1, x.dim() + 1):
        if ds[:k] == tuple(x.shape[:k]) and all(d == 1 for d in ds[k:]):
            return x.numel() // nd, nd
    raise ValueError(f"unsupported delta shape {tuple(delta.shape)} for x {tuple(x.shape)}")


def _zp_like(zp, delta):
    """Expand a per-row zero point to delta's per-(row, in-channel) layout if needed."""
    if zp.numel() == delta.numel() or zp.numel() == 1 and delta.numel() == 1:
        return zp
    return zp.expand(delta.shape).contiguous() if zp.dim() == delta.dim() else \
        zp.reshape(zp.shape + (1,) * (delta.dim() - zp.dim())).expand(delta.shape).contiguous()


def fake_quant_fwd(x, delta, zp, n_bits, sym=False, scale=1.0, codes=False, out=None,
                   ste=True):
    """UniformAffineQuantizer.forward (quant_layer.py:92-98). Returns (y, codes|None);
    `out` (same shape, fp32, on the device) receives y when given.  ste=True rounds as the
    reference's round_ste ((round(t) - t) + t: NaN at t = +-inf), ste=False as plain
    torch.round (ChannelQuant / ChannelQuantAct 'none', AdaRound 'nearest')."""
    x, xp = fptr(x, "x")
    delta, dp = fptr(delta.detach(), "delta")
    zp, zpp = fptr(_zp_like(zp.detach(), delta), "zero_point")
    inner, nch = _channel_layout(x, delta)
    lo, hi = qrange(n_bits, sym)
    if out is not None:
        y, _ = fptr(out, "out")
        if y.shape != x.shape or y is not out:
            raise A.SSQError("fake_quant_fwd: out must be a contiguous tensor shaped like x")
    else:
        y = torch.empty_like(x)
    cb = _codes_buf(x, codes)
    call("ssq_fq_fwd" if ste else "ssq_fq_round_fwd", xp, _vp(y), _vp(cb), dp, zpp, x.numel(),
         inner, nch, float(scale), lo, hi, stream_of(x))
    return y, cb


class FakeQuantFn(torch.autograd.Function):
    """round_ste fake-quant with the reference's autograd: STE for x, exact chain for
    delta / zero_point (used by the act-delta LSQ recon, block_recon.py:62-73)."""

    @staticmethod
    def forward(ctx, x, delta, zp, n_bits, sym):
        y, _ = fake_quant_fwd(x, delta, zp, n_bits, sym)
        ctx.save_for_backward(x, delta, zp)
        ctx.q = (n_bits, sym)
        return y

    @staticmethod
    def backward(ctx, gy):
        x, delta, zp = ctx.saved_tensors
        n_bits, sym = ctx.q
        x = x.contiguous()
        gy = gy.contiguous()
        d, z = delta.detach().contiguous(), zp.detach().contiguous()
        inner, nch = _channel_layout(x, d)
        lo, hi = qrange(n_bits, sym)
        need_x, need_d, need_z = ctx.needs_input_grad[0], ctx.needs_input_grad[1], ctx.needs_input_grad[2]
        gx = torch.empty_like(x) if need_x else None
        gd = torch.empty(d.numel(), dtype=torch.float32, device=x.device) if need_d else None
        gz = torch.empty(z.numel(), dtype=torch.float32, device=x.device) if need_z else None
        wsb = query("ssq_fq_bwd_workspace_size", x.numel(), inner, nch)
        ws, wsn = workspace(wsb, x.device)
        call("ssq_fq_bwd", _vp(x), _vp(gy), _vp(d), _vp(z), x.numel(), inner, nch, lo, hi,
             _vp(gx), _vp(gd), _vp(gz), ws, wsn, stream_of(x))
        return (gx, None if gd is None else gd.view(delta.shape),
                None if gz is None else gz.view(zp.shape), None, None)


def fake_quant(x, delta, zp, n_bits, sym=False):
    return FakeQuantFn.apply(x, delta, zp, n_bits, sym)


class RoundQuantFn(torch.autograd.Function):
    """q/dq with torch.round (NO straight-through estimator) at delta*scale, clamp
    [lo, hi]: ChannelQuantAct 'none' mode (channelQuantAct.py:56-67).  The reference's
    autograd gives d/dx = 0 (round has a zero gradient), d/ddelta = scale * sum g*(q-zp)
    (through the product delta*shiftedScale), d/dzp = -sum_{clamped} g*delta*scale."""

    @staticmethod
    def forward(ctx, x, delta, zp, n_bits, sym, scale):
        y, _ = fake_quant_fwd(x, delta, zp, n_bits, sym, scale=scale, ste=False)
        ctx.save_for_backward(x, delta, zp)
        ctx.q = (n_bits, sym, scale)
        return y

    @staticmethod
    def backward(ctx, gy):
        x, delta, zp = ctx.saved_tensors
        n_bits, sym, scale = ctx.q
        need_x, need_d, need_z = ctx.needs_input_grad[:3]
        gx = torch.zeros_like(x) if need_x else None
        if not (need_d or need_z):
            return gx, None, None, None, None, None
        x, gy = x.contiguous(), gy.contiguous()
        # the product delta*shiftedScale as the reference forms it (tensor * python float)
        t = (delta.detach() * scale).contiguous()
        z = _zp_like(zp.detach(), t).contiguous()
        inner, nch = _channel_layout(x, t)
        lo, hi = qrange(n_bits, sym)
        gt = torch.empty(t.numel(), dtype=torch.float32, device=x.device)
        gz = torch.empty(z.numel(), dtype=torch.float32, device=x.device) if need_z else None
        wsb = query("ssq_fq_bwd_workspace_size", x.numel(), inner, nch)
        ws, wsn = workspace(wsb, x.device)
        call("ssq_fq_round_bwd", _vp(x), _vp(gy), _vp(t), _vp(z), x.numel(), inner, nch, lo, hi,
             _vp(gt), _vp(gz), ws, wsn, stream_of(x))
        gd = (gt * scale).view(delta.shape) if need_d else None
        return (gx, gd, None if gz is None else gz.view(zp.shape), None, None, None)


def round_quant(x, delta, zp, n_bits, sym=False, scale=1.0):
    return RoundQuantFn.apply(x, delta, zp, n_bits, sym, float(scale))


class FqMultiPlan:
    """fake_quant_multi's arguments checked and packed once: calling the plan launches the
    same table again (one ctypes call), e.g. a fixed model's weights quantised every step.
    The plan holds its tensors and reads their current values at each launch, so in-place
    updates of x / delta / zero_point are seen; it therefore refuses non-contiguous inputs
    (a contiguous copy would freeze their values at plan time).  A tensor replaced by a new
    one needs a new plan.  fake_quant_multi (one launch) copies non-contiguous inputs."""

    def __init__(self, xs, deltas, zps, n_bits, sym=False, out=None, _once=False):
        n = len(xs)
        if not _once:
            for k, (x, d, z) in enumerate(zip(xs, deltas, zps)):
                for t, what in ((x, "x"), (d, "delta"), (z, "zero_point")):
                    if not t.is_contiguous():
                        raise ValueError(f"FqMultiPlan: {what}[{k}] is not contiguous (a copy "
                                         "would not see later in-place updates)")
        if out is None:
            ys = [torch.empty_like(x) for x in xs]
        else:
            if len(out) != n:
                raise ValueError(f"fake_quant_multi: {len(out)} outputs for {n} inputs")
            for k, (x, y) in enumerate(zip(xs, out)):
                A.check(y, f"out[{k}]")
                if y.shape != x.shape or not y.is_contiguous():
                    raise ValueError(f"fake_quant_multi: out[{k}] must be contiguous, shape "
                                     f"{tuple(x.shape)}")
            ys = list(out)
        keep = []
        P = C.c_void_p * n
        xa, ya, da, za = P(), P(), P(), P()
        na, ia, ca = (C.c_int64 * n)(), (C.c_int64 * n)(), (C.c_int64 * n)()
        lo_a, hi_a = (C.c_int * n)(), (C.c_int * n)()
        nb = n_bits if isinstance(n_bits, (list, tuple)) else [n_bits] * n
        for k, (x, d, z, y) in enumerate(zip(xs, deltas, zps, ys)):
            x, xp = fptr(x)
            d, dp = fptr(d.detach())
            z, zpp = fptr(z.detach())
            keep += [x, d, z]
            inner, nch = _channel_layout(x, d)
            xa[k], ya[k], da[k], za[k] = xp.value, y.data_ptr(), dp.value, zpp.value
            na[k], ia[k], ca[k] = x.numel(), inner, nch
            lo_a[k], hi_a[k] = qrange(nb[k], sym)
        self.ys, self.keep = ys, keep
        self.args = (n, xa, ya, da, za, na, ia, ca, lo_a, hi_a)
        self.device = xs[0].device

    def __call__(self):
        call("ssq_fq_fwd_multi", *self.args, stream_of(self.ys[0]))
        if _DEFERRED_FQ_KEEP is not None:
            # the table may launch later (riding on the next per-tensor launch): keep any
            # contiguous copies made for it alive until then
            _DEFERRED_FQ_KEEP.append(self)
        return self.ys


def fake_quant_multi(xs, deltas, zps, n_bits, sym=False, out=None):
    """Every tensor of a list in one launch (per-channel params staged in LDS); out: a
    list of contiguous fp32 outputs, one per input and of its shape (else allocated).
    FqMultiPlan packs the same arguments once for repeated launches."""
    return FqMultiPlan(xs, deltas, zps, n_bits, sym, out, _once=True)()


_DEFERRED_FQ_KEEP = None


def maxpool2d(x, k, stride, padding):
    """F.max_pool2d forward (no dilation, floor mode) on ssq_maxpool2d_fwd: bit-identical to
    torch's, NCHW fp32 on the device, K <= 7, padding <= K // 2."""
    x, xp = fptr(x, "x")
    N, C_, H, W = (int(v) for v in x.shape)
    OH, OW = (H + 2 * padding - k) // stride + 1, (W + 2 * padding - k) // stride + 1
    y = torch.empty((N, C_, OH, OW), dtype=torch.float32, device=x.device)
    call("ssq_maxpool2d_fwd", xp, _vp(y), N, C_, H, W, int(k), int(stride), int(padding),
         stream_of(x))
    return y


# QuantModel swaps nn.MaxPool2d for SsqMaxPool2d (A/B knob: SSQ_MAXPOOL=0 keeps torch's)
MAXPOOL_HIP = os.environ.get("SSQ_MAXPOOL", "1") != "0"


class SsqMaxPool2d(torch.nn.MaxPool2d):
    """nn.MaxPool2d whose forward runs on ssq_maxpool2d_fwd where it applies (a square
    window of <= 7, padding <= K // 2, no dilation / ceil mode / indices, a 4-D fp32 device
    input that needs no gradient); torch's pooling otherwise.  Same results either way."""

    @staticmethod
    def wrap(m):
        s = SsqMaxPool2d(m.kernel_size, m.stride, m.padding, m.dilation, m.return_indices,
                         m.ceil_mode)
        return s

    def _plan(self):
        def one(v):
            if isinstance(v, int):
                return v
            return v[0] if len(set(v)) == 1 else None
        k, st, pad, dil = (one(v) for v in (self.kernel_size, self.stride, self.padding,
                                            self.dilation))
        if None in (k, st, pad, dil) or dil != 1 or self.ceil_mode or self.return_indices:
            return None
        if k > 7 or 2 * pad > k:
            return None
        return k, st, pad

    def forward(self, x):
        plan = self._plan()
        if (plan is not None and x.dim() == 4 and x.is_cuda and x.dtype == torch.float32
                and not (torch.is_grad_enabled() and x.requires_grad)):
            return maxpool2d(x, *plan)
        return super().forward(x)


class deferred_fq_multi:
    """Context: a fake_quant_multi inside it rides on the next per-tensor fake_quant_fwd of
    its stream -- one launch for both (include/ssq.h ssq_set_deferred_fq_multi); a table
    still queued at exit is launched then."""

    def __init__(self, on=True, device=None):
        self.on, self.device = on, device

    def __enter__(self):
        global _DEFERRED_FQ_KEEP
        self.prev = bool(query("ssq_set_deferred_fq_multi", 1)) if self.on else None
        if self.on:
            self.prev_keep, _DEFERRED_FQ_KEEP = _DEFERRED_FQ_KEEP, []
        return self

    def __exit__(self, *exc):
        global _DEFERRED_FQ_KEEP
        if self.on:
            dev_ = torch.device("cuda", torch.cuda.current_device()) if self.device is None \
                else self.device
            try:
                call("ssq_flush_fq_multi", C.c_void_p(torch.cuda.current_stream(dev_).cuda_stream))
            finally:
                query("ssq_set_deferred_fq_multi", int(self.prev))
                # every queued table has launched: its inputs may be freed (stream order)
                _DEFERRED_FQ_KEEP = self.prev_keep


# ------------------------------------------------------------------ K3/K4
class ScaleInitError(A.SSQError, ValueError):
    """A row the reference's init_quantization_scale cannot initialise."""


def scale_init(x, n_bits, sym=False, channel_wise=False, method="max", return_scores=False,
               check=True):
    """init_quantization_scale (quant_layer.py:100-166) on the device.
    Returns (delta, zero_point, raw_zero_point) shaped like the reference's:
    (Co,1,1,1)/(Co,1) for channel_wise, 0-dim otherwise.

    A row holding NaN (or, for 'max', -inf; for 'mse', any infinity or a constant row) has no
    init in the reference: 'max' raises ValueError at round(nan) (:140), 'mse' never assigns
    delta (:147-162) and fails where it is used.  ssq_scale_init marks such rows NaN and this
    raises ScaleInitError (an SSQError and a ValueError) naming them -- one host sync, as the
    reference's own .item() calls; check=False skips it (the caller inspects the NaN rows)."""
    x, xp = fptr(x.detach(), "x")
    if "max" in method:
        m, sflag = 0, int("scale" in method)
    elif method == "mse":
        m, sflag = 1, 0
    else:
        raise NotImplementedError(method)
    rows = x.shape[0] if channel_wise else 1
    inner = x.numel() // rows
    d = torch.empty(rows, dtype=torch.float32, device=x.device)
    z = torch.empty_like(d)
    r = torch.empty_like(d)
    sc = torch.empty(rows, 80, dtype=torch.float64, device=x.device) if (return_scores and m == 1) else None
    wsb = query("ssq_scale_init_workspace_size", rows, inner, m)
    ws, wsn = workspace(wsb, x.device)
    call("ssq_scale_init", xp, rows, inner, n_bits, int(sym), m, sflag, _vp(d), _vp(z), _vp(r),
         _vp(sc), ws, wsn, stream_of(x))
    if check:
        bad = torch.isnan(d) | torch.isnan(z)
        if bool(bad.any()):
            rows_bad = bad.nonzero().flatten()[:8].tolist()
            raise ScaleInitError(f"ssq_scale_init ({method}): {int(bad.sum())} of {rows} rows have "
                                 f"no quantization scale (NaN / infinite input; rows {rows_bad}...), "
                                 f"as the reference's init_quantization_scale raises there")
    if channel_wise:
        shape = (-1,) + (1,) * (x.dim() - 1)
        out = d.view(shape), z.view(shape), r.view(shape)
    else:
        out = d.view(()), z.view(()), r.view(())
    return out + (sc,) if return_scores else out


# ------------------------------------------------------------------ K9 inits
def shift_init(w, delta, shifts, zp=None, n_bits=None, sym=False, mode=0):
    """ChannelQuant.init_v_beta (mode 0, channelQuant.py:279-294) -> (alpha, beta, mse) or
    init_v's alpha (mode 1, channelQuant.py:201-213; beta is None)."""
    w, wp = fptr(w.detach(), "weight")
    delta, dp = fptr(delta.detach(), "delta")
    z, zpp = fptr(zp.detach(), "zero_point") if zp is not None else (None, None)
    Co, Ci, K, is_fc = geometry(w)
    S = len(shifts)
    lo, hi = qrange(n_bits, sym) if mode == 1 else (0, 1)
    alpha = torch.empty((Co, Ci, S) if is_fc else (Ci, S), dtype=torch.float32, device=w.device)
    mse = torch.empty_like(alpha)
    beta = torch.empty_like(w) if mode == 0 else None
    wsb = query("ssq_shift_init_workspace_size", Co, Ci, K, S, is_fc)
    ws, wsn = workspace(wsb, w.device)
    call("ssq_shift_init", wp, dp, zpp, A.shifts_arg(shifts), S, Co, Ci, K, is_fc, int(mode), lo, hi,
         _vp(alpha), _vp(beta), _vp(mse), ws, wsn, stream_of(w))
    return alpha, beta, mse


def rect_init(w, delta):
    """beta = -log((zeta-gamma)/(rest-gamma) - 1) (channelQuant.py:300-307,
    adaptive_rounding.py:72-78); delta per output row or per (row, in-channel)."""
    w, wp = fptr(w.detach(), "weight")
    delta, dp = fptr(delta.detach(), "delta")
    Co, Ci, K, _ = geometry(w)
    per_ci = _delta_per_ci(delta, Co, Ci)
    beta = torch.empty_like(w)
    call("ssq_rect_init", wp, dp, per_ci, Co, Ci, K, _vp(beta), stream_of(w))
    return beta


def _delta_per_ci(delta, Co, Ci):
    if delta.numel() == Co:
        return 0
    if delta.numel() == Co * Ci:
        return 1
    raise ValueError(f"delta with {delta.numel()} entries for ({Co},{Ci}) weight")


def get_delta(delta, alpha, shifts, w_shape):
    """ChannelQuant.get_delta (channelQuant.py:221-237) -> (Co,Ci,1,1) conv / (Co,Ci) fc."""
    delta, dp = fptr(delta.detach(), "delta")
    alpha, ap = fptr(alpha.detach(), "alpha")
    Co, Ci = int(w_shape[0]), int(w_shape[1])
    is_fc = int(len(w_shape) == 2)
    out = torch.empty(Co, Ci, dtype=torch.float32, device=delta.device)
    call("ssq_get_delta", dp, ap, A.shifts_arg(shifts), len(shifts), Co, Ci, is_fc, _vp(out),
         stream_of(delta))
    return out if is_fc else out.view(Co, Ci, 1, 1)


# ------------------------------------------------------------------ K5/K6 adaShift
class AdaShiftFn(torch.autograd.Function):
    """ChannelQuant.forward 'adaShift' (channelQuant.py:51-64).  Gradients flow to alpha
    (soft targets only) and beta (soft rounding only), as in the reference's autograd.
    `reg` = (lambda, b, reg_vals, reg_dev) optionally fuses the shift regulariser: its
    gradient is added to alpha's inside the same backward kernel, (lambda, b) taken from
    the device pair reg_dev when given (graph-capturable)."""

    @staticmethod
    def forward(ctx, alpha, beta, w, delta, zp, shifts, n_bits, sym, hard_t, hard_r, reg):
        w, wp = fptr(w.detach(), "weight")
        a, ap = fptr(alpha.detach(), "alpha")
        b, bp = fptr(beta.detach(), "beta")
        d, dp = fptr(delta.detach(), "delta")
        z, zpp = fptr(zp.detach(), "zero_point")
        Co, Ci, K, is_fc = geometry(w)
        lo, hi = qrange(n_bits, sym)
        out = torch.empty_like(w)
        call("ssq_adashift_fwd", wp, ap, bp, dp, zpp, A.shifts_arg(shifts), len(shifts), Co, Ci, K,
             is_fc, int(hard_t), int(hard_r), lo, hi, _vp(out), None, stream_of(w))
        ctx.save_for_backward(a, b, w, d, z)
        ctx.cfg = (tuple(shifts), n_bits, sym, hard_t, hard_r, reg)
        return out

    @staticmethod
    def backward(ctx, g):
        a, b, w, d, z = ctx.saved_tensors
        shifts, n_bits, sym, hard_t, hard_r, reg = ctx.cfg
        need_a = ctx.needs_input_grad[0] and not hard_t
        need_b = ctx.needs_input_grad[1] and not hard_r
        if not (need_a or need_b):
            return (None,) * 11
        g = g.contiguous()
        Co, Ci, K, is_fc = geometry(w)
        lo, hi = qrange(n_bits, sym)
        ga = torch.empty_like(a)
        gb = torch.empty_like(w) if need_b else None
        lam, bb, reg_vals, reg_dev = (0.0, 0.0, None, None) if reg is None else reg
        S = len(shifts)
        wsb = query("ssq_adashift_bwd_workspace_size", Co, Ci, K, S, is_fc)
        ws, wsn = workspace(wsb, w.device)
        call("ssq_adashift_bwd", _vp(g), _vp(w), _vp(a), _vp(b), _vp(d), _vp(z),
             A.shifts_arg(shifts), S, Co, Ci, K, is_fc, int(hard_r), lo, hi, float(lam), float(bb),
             _vp(reg_dev), _vp(ga), _vp(gb), _vp(reg_vals), ws, wsn, stream_of(w))
        return (ga if need_a else None, gb, None, None, None, None, None, None, None, None, None)


def adashift(alpha, beta, w, delta, zp, shifts, n_bits, sym, hard_t, hard_r, reg=None):
    return AdaShiftFn.apply(alpha, beta, w, delta, zp, tuple(shifts), n_bits, sym, bool(hard_t),
                            bool(hard_r), reg)


class AdaShiftPrep:
    """Loop-invariant state of a conv ChannelQuant in 'adaShift' mode (W, delta, shifts,
    beta frozen, as in the fused loop): the packed int8 floors and h(beta) of
    ssq_adashift_prepare.  `ok` is False when a floor does not fit int8 or the kernel
    window exceeds 256 taps (the caller keeps the recomputing kernels)."""

    def __init__(self, w, beta, delta, shifts, hard_r):
        w, wp = fptr(w.detach(), "weight")
        b, bp = fptr(beta.detach(), "beta")
        d, dp = fptr(delta.detach(), "delta")
        Co, Ci, K, is_fc = geometry(w)
        if is_fc:
            raise A.SSQError("AdaShiftPrep: conv weights only")
        self.geo = (Co, Ci, K)
        self.S = len(shifts)
        self.fpack = torch.empty(w.shape, dtype=torch.int32, device=w.device)
        self.hterm = torch.empty_like(w)
        flag = torch.zeros(1, dtype=torch.int32, device=w.device)
        call("ssq_adashift_prepare", wp, bp, dp, A.shifts_arg(shifts), self.S, Co, Ci, K,
             int(hard_r), _vp(self.fpack), _vp(self.hterm), _vp(flag), stream_of(w))
        self.ok = int(flag.item()) == 0 and K <= 256   # one sync, at preparation time only


def _ptrs(ts):
    return (C.c_void_p * len(ts))(*[None if t is None else t.data_ptr() for t in ts])


# Gradient destinations of leaf parameters (data_ptr -> contiguous tensor of the parameter's
# size), set by the data-parallel loop to the slices of its all-reduce bucket (grads_into):
# the backward kernels below then write a parameter's gradient straight into its slice and
# hand autograd None for it -- no AccumulateGrad add, and a deferred finalize (fin_tasks.h)
# may still be pending when backward returns: nothing reads the slice before the collective,
# which runs after the iteration's queued finalizes are flushed.  Each such parameter must
# get its gradient from exactly one kernel per iteration (alpha: its adaShift backward;
# gamma^z / phi^z: their module's epilogue).
GRAD_INTO = {}
INTO_WRITES = [0]       # gradients written straight into a GRAD_INTO slice (test counter)
_INTO_SEEN = set()      # the parameters already written into inside the current context


class grads_into:
    """Context: GRAD_INTO = mapping (param.data_ptr() -> destination) inside.  One context
    spans one iteration's backward: a second kernel producing the same parameter's gradient
    inside it would overwrite the first's contribution instead of adding to it, so it
    raises SSQError instead."""

    def __init__(self, mapping):
        self.mapping = mapping or {}

    def __enter__(self):
        self.prev = dict(GRAD_INTO), set(_INTO_SEEN)
        GRAD_INTO.clear()
        GRAD_INTO.update(self.mapping)
        _INTO_SEEN.clear()
        return self

    def __exit__(self, *exc):
        GRAD_INTO.clear()
        GRAD_INTO.update(self.prev[0])
        _INTO_SEEN.clear()
        _INTO_SEEN.update(self.prev[1])


def _grad_dest(param, numel, device, need=True):
    """(destination tensor, written_into) for a parameter's gradient: its GRAD_INTO slice,
    or a fresh buffer (None when the gradient is not needed)."""
    if param is None or not need:
        return None, False
    d = GRAD_INTO.get(param.data_ptr()) if GRAD_INTO else None
    if d is not None:
        if d.numel() != numel or not d.is_contiguous():
            raise A.SSQError("grads_into: destination does not match the parameter")
        if param.data_ptr() in _INTO_SEEN:
            raise A.SSQError("grads_into: a second kernel produces the gradient of the same "
                             "parameter in one iteration (it would overwrite, not add)")
        _INTO_SEEN.add(param.data_ptr())
        INTO_WRITES[0] += 1
        return d.view(-1), True
    return torch.empty(numel, device=device), False


class AdaShiftPrepFn(torch.autograd.Function):
    """ChannelQuant 'adaShift' forward of SEVERAL prepared weights (e.g. every conv of a
    block, same S and regulariser) in one launch (K5p), and their alpha backward in two
    (K6p, shift regulariser folded in as in AdaShiftFn).  cfg = (hard_t, reg, entries),
    entries[i] = (prep, delta, zp, n_bits, sym); inputs = the alphas; outputs = the Whats."""

    @staticmethod
    def forward(ctx, cfg, *alphas):
        hard_t, reg, entries = cfg
        keep, al, dl, zl = [], [], [], []
        for a, (prep, d, z, n_bits, sym) in zip(alphas, entries):
            a, _ = fptr(a.detach(), "alpha")
            d, _ = fptr(d.detach(), "delta")
            z, _ = fptr(z.detach(), "zero_point")
            al.append(a)
            dl.append(d)
            zl.append(z)
        n = len(entries)
        preps = [e[0] for e in entries]
        outs = [torch.empty_like(p.hterm) for p in preps]
        Co = (C.c_int64 * n)(*[p.geo[0] for p in preps])
        Ci = (C.c_int64 * n)(*[p.geo[1] for p in preps])
        Kk = (C.c_int64 * n)(*[p.geo[2] for p in preps])
        qr = [qrange(e[3], e[4]) for e in entries]
        lo = (C.c_int * n)(*[q[0] for q in qr])
        hi = (C.c_int * n)(*[q[1] for q in qr])
        call("ssq_adashift_fwd_prepared_multi", n, _ptrs([p.fpack for p in preps]),
             _ptrs([p.hterm for p in preps]), _ptrs(al), _ptrs(dl), _ptrs(zl), Co, Ci, Kk, lo, hi,
             preps[0].S, int(hard_t), _ptrs(outs), stream_of(outs[0]))
        ctx.save_for_backward(*al, *dl, *zl)
        ctx.cfg = (hard_t, reg, preps, (Co, Ci, Kk, lo, hi))
        return tuple(outs)

    @staticmethod
    def backward(ctx, *gs):
        hard_t, reg, preps, (Co, Ci, Kk, lo, hi) = ctx.cfg
        n = len(preps)
        if hard_t or not any(ctx.needs_input_grad[1:]):
            return (None,) * (n + 1)
        saved = ctx.saved_tensors
        al, dl, zl = saved[:n], saved[n:2 * n], saved[2 * n:]
        gs = [torch.zeros_like(p.hterm) if g is None else g.contiguous() for g, p in zip(gs, preps)]
        dst = [_grad_dest(a, a.numel(), a.device) for a in al]
        gas = [d.view(a.shape) for (d, _), a in zip(dst, al)]
        lam, bb, reg_vals, reg_dev = (0.0, 0.0, None, None) if reg is None else reg
        rv = reg_vals if isinstance(reg_vals, (list, tuple)) else [reg_vals] * n
        S = preps[0].S
        wsb = query("ssq_adashift_bwd_prepared_multi_workspace_size", n, Co, Ci, Kk, S)
        ws, wsn = workspace(wsb, gs[0].device)
        call("ssq_adashift_bwd_prepared_multi", n, _ptrs(gs), _ptrs([p.fpack for p in preps]),
             _ptrs([p.hterm for p in preps]), _ptrs(al), _ptrs(dl), _ptrs(zl), Co, Ci, Kk, lo, hi, S,
             float(lam), float(bb), _vp(reg_dev), _ptrs(gas),
             _ptrs(rv) if any(v is not None for v in rv) else None, ws, wsn, stream_of(gs[0]))
        return (None,) + tuple(ga if (need and not into) else None
                               for ga, (_, into), need in zip(gas, dst, ctx.needs_input_grad[1:]))


def adashift_prepared(alpha, prep, delta, zp, n_bits, sym, hard_t, reg=None):
    """One prepared weight (ChannelQuant.forward in 'adaShift' mode)."""
    return AdaShiftPrepFn.apply((bool(hard_t), reg, ((prep, delta, zp, n_bits, sym),)), alpha)[0]


def adashift_prepared_multi(alphas, entries, hard_t, reg=None):
    """Several prepared weights (same S, same regulariser schedule) in one launch."""
    return AdaShiftPrepFn.apply((bool(hard_t), reg, tuple(entries)), *alphas)


def adashift_codes(alpha, beta, w, delta, zp, shifts, n_bits, sym):
    """Hard/hard adaShift: dequantized weight and the integer codes (uint8/int8)."""
    w, wp = fptr(w.detach())
    a, ap = fptr(alpha.detach())
    b, bp = fptr(beta.detach())
    d, dp = fptr(delta.detach())
    z, zpp = fptr(zp.detach())
    Co, Ci, K, is_fc = geometry(w)
    lo, hi = qrange(n_bits, sym)
    out = torch.empty_like(w)
    codes = torch.empty(w.shape, dtype=torch.uint8, device=w.device)
    call("ssq_adashift_fwd", wp, ap, bp, dp, zpp, A.shifts_arg(shifts), len(shifts), Co, Ci, K,
         is_fc, 1, 1, lo, hi, _vp(out), _vp(codes), stream_of(w))
    return out, (codes.view(torch.int8) if sym else codes)


# ------------------------------------------------------------------ K7 learned_hard_sigmoid
class LhsFn(torch.autograd.Function):
    """ChannelQuant 'learned_hard_sigmoid' (channelQuant.py:81-82, :96-118) with the
    dequantized candidates of init_v (channelQuant.py:201-213) recomputed in-kernel."""

    @staticmethod
    def forward(ctx, alpha, w, delta, zp, shifts, n_bits, sym, hard_t):
        w, wp = fptr(w.detach())
        a, ap = fptr(alpha.detach())
        d, dp = fptr(delta.detach())
        z, zpp = fptr(zp.detach())
        Co, Ci, K, is_fc = geometry(w)
        lo, hi = qrange(n_bits, sym)
        out = torch.empty_like(w)
        call("ssq_lhs_fwd", wp, ap, dp, zpp, A.shifts_arg(shifts), len(shifts), Co, Ci, K, is_fc,
             int(hard_t), lo, hi, _vp(out), stream_of(w))
        ctx.save_for_backward(a, w, d, z)
        ctx.cfg = (tuple(shifts), n_bits, sym, hard_t)
        return out

    @staticmethod
    def backward(ctx, g):
        a, w, d, z = ctx.saved_tensors
        shifts, n_bits, sym, hard_t = ctx.cfg
        if hard_t or not ctx.needs_input_grad[0]:
            return (None,) * 8
        g = g.contiguous()
        Co, Ci, K, is_fc = geometry(w)
        lo, hi = qrange(n_bits, sym)
        ga = torch.empty_like(a)
        S = len(shifts)
        wsb = query("ssq_adashift_bwd_workspace_size", Co, Ci, K, S, is_fc)
        ws, wsn = workspace(wsb, w.device)
        call("ssq_lhs_bwd", _vp(g), _vp(w), _vp(a), _vp(d), _vp(z), A.shifts_arg(shifts), S, Co, Ci,
             K, is_fc, lo, hi, _vp(ga), ws, wsn, stream_of(w))
        return (ga, None, None, None, None, None, None, None)


def lhs(alpha, w, delta, zp, shifts, n_bits, sym, hard_t):
    return LhsFn.apply(alpha, w, delta, zp, tuple(shifts), n_bits, sym, bool(hard_t))


# ------------------------------------------------------------------ K8 adaround
class AdaRoundFn(torch.autograd.Function):
    """floor(W/d) + h(beta) (soft) or [beta>=0] (hard), clamp, dequant
    (channelQuant.py:65-78, adaptive_rounding.py:55-67)."""

    @staticmethod
    def forward(ctx, beta, w, delta, zp, n_bits, sym, hard_r, scale, reg=None):
        w, wp = fptr(w.detach())
        b, bp = fptr(beta.detach())
        d, dp = fptr(delta.detach())
        z, zpp = fptr(zp.detach())
        Co, Ci, K, _ = geometry(w)
        per_ci = _delta_per_ci(d, Co, Ci)
        lo, hi = qrange(n_bits, sym)
        out = torch.empty_like(w)
        call("ssq_adaround_fwd", wp, bp, dp, per_ci, zpp, float(scale), Co, Ci, K, int(hard_r), lo,
             hi, _vp(out), None, stream_of(w))
        ctx.save_for_backward(b, w, d, z)
        ctx.cfg = (n_bits, sym, hard_r, scale, per_ci, reg)
        return out

    @staticmethod
    def backward(ctx, g):
        b, w, d, z = ctx.saved_tensors
        n_bits, sym, hard_r, scale, per_ci, reg = ctx.cfg
        if hard_r or not ctx.needs_input_grad[0]:
            return (None,) * 9
        g = g.contiguous()
        Co, Ci, K, _ = geometry(w)
        lo, hi = qrange(n_bits, sym)
        gb = torch.empty_like(w)
        lam, bb, reg_dev = (0.0, 0.0, None) if reg is None else reg
        call("ssq_adaround_bwd", _vp(g), _vp(w), _vp(b), _vp(d), per_ci, _vp(z), float(scale), Co,
             Ci, K, lo, hi, float(lam), float(bb), _vp(reg_dev), _vp(gb), stream_of(w))
        return (gb, None, None, None, None, None, None, None, None)


class AdaRoundMultiFn(torch.autograd.Function):
    """AdaRoundFn for several weights (a block's AdaRound quantizers) in one launch each way
    (ssq_adaround_fwd_multi / _bwd_multi; bit-identical to one launch per weight).
    cfg = (hard_r, reg, entries), entries[i] = (w, delta, zp, n_bits, sym, scale); inputs =
    the betas; outputs = the Whats."""

    @staticmethod
    def forward(ctx, cfg, *betas):
        hard_r, reg, entries = cfg
        n = len(entries)
        ws, bs, ds, zs, outs, geo, pc, sc, lo_, hi_ = [], [], [], [], [], [], [], [], [], []
        for b, (w, d, z, n_bits, sym, scale) in zip(betas, entries):
            w, _ = fptr(w.detach(), "weight")
            b, _ = fptr(b.detach(), "beta")
            d, _ = fptr(d.detach(), "delta")
            z, _ = fptr(z.detach(), "zero_point")
            Co, Ci, K, _ = geometry(w)
            ws.append(w)
            bs.append(b)
            ds.append(d)
            zs.append(z)
            outs.append(torch.empty_like(w))
            geo.append((Co, Ci, K))
            pc.append(_delta_per_ci(d, Co, Ci))
            sc.append(float(scale))
            lo, hi = qrange(n_bits, sym)
            lo_.append(lo)
            hi_.append(hi)
        arr = (C.c_int64 * n)
        args = (arr(*[g[0] for g in geo]), arr(*[g[1] for g in geo]), arr(*[g[2] for g in geo]))
        ints = ((C.c_int * n)(*pc), (C.c_float * n)(*sc), (C.c_int * n)(*lo_), (C.c_int * n)(*hi_))
        call("ssq_adaround_fwd_multi", n, _ptrs(ws), _ptrs(bs), _ptrs(ds), ints[0], _ptrs(zs),
             ints[1], *args, int(hard_r), ints[2], ints[3], _ptrs(outs), stream_of(ws[0]))
        ctx.save_for_backward(*bs, *ws, *ds, *zs)
        ctx.cfg = (hard_r, reg, n, args, ints)
        return tuple(outs)

    @staticmethod
    def backward(ctx, *gs):
        hard_r, reg, n, args, ints = ctx.cfg
        if hard_r or not any(ctx.needs_input_grad[1:]):
            return (None,) * (n + 1)
        saved = ctx.saved_tensors
        bs, ws, ds, zs = saved[:n], saved[n:2 * n], saved[2 * n:3 * n], saved[3 * n:]
        gs = [torch.zeros_like(w) if g is None else g.contiguous() for g, w in zip(gs, ws)]
        gb = [torch.empty_like(w) for w in ws]
        lam, bb, reg_dev = (0.0, 0.0, None) if reg is None else reg
        call("ssq_adaround_bwd_multi", n, _ptrs(gs), _ptrs(ws), _ptrs(bs), _ptrs(ds), ints[0],
             _ptrs(zs), ints[1], *args, ints[2], ints[3], float(lam), float(bb), _vp(reg_dev),
             _ptrs(gb), stream_of(ws[0]))
        return (None,) + tuple(g if need else None for g, need in zip(gb, ctx.needs_input_grad[1:]))


def adaround_multi(betas, entries, hard_r, reg=None):
    """Several AdaRound weights in one launch (AdaRoundMultiFn)."""
    return AdaRoundMultiFn.apply((bool(hard_r), reg, tuple(entries)), *betas)


def adaround(beta, w, delta, zp, n_bits, sym, hard_r, scale=1.0, reg=None):
    """reg = (lambda, b, reg_dev) folds the rounding regulariser's gradient into the
    backward ((lambda, b) from the device pair reg_dev when given)."""
    return AdaRoundFn.apply(beta, w, delta, zp, n_bits, sym, bool(hard_r), float(scale), reg)


# ------------------------------------------------------------------ K12 regularisers
class ShiftRegFn(torch.autograd.Function):
    """lambda*sum(1-|2p-1|^b) (mode 0) or lambda*-sum p log(p+1e-10) (mode 1) of
    p = get_sig_soft_targets(alpha) (layer_recon_fused_shiftedScale.py:281-282,
    layer_recon_shiftedScale.py:393)."""

    @staticmethod
    def forward(ctx, alpha, lam, b, mode):
        a, ap = fptr(alpha.detach())
        S = a.shape[-1]
        rows = a.numel() // S
        vals = torch.empty(rows, dtype=torch.float32, device=a.device)
        call("ssq_shift_reg", ap, S, rows, int(mode), float(lam), float(b), None, _vp(vals),
             stream_of(a))
        ctx.save_for_backward(a)
        ctx.cfg = (lam, b, mode)
        return vals.sum()

    @staticmethod
    def backward(ctx, g):
        (a,) = ctx.saved_tensors
        lam, b, mode = ctx.cfg
        S = a.shape[-1]
        ga = torch.zeros_like(a)
        call("ssq_shift_reg", _vp(a), S, a.numel() // S, int(mode), float(lam), float(b), _vp(ga),
             None, stream_of(a))
        return ga * g, None, None, None


def shift_reg(alpha, lam, b, mode=0):
    return ShiftRegFn.apply(alpha, lam, b, mode)


class RoundRegFn(torch.autograd.Function):
    """lambda*sum(1-|2h(v)-1|^b) with h the rectified sigmoid (block_recon.py:171-174,
    layer_recon_fused_shiftedScale.py:278-279)."""

    @staticmethod
    def forward(ctx, v, lam, b):
        v, vp = fptr(v.detach())
        loss = torch.empty(1, dtype=torch.float32, device=v.device)
        ws, wsn = workspace(query("ssq_round_reg_workspace_size", v.numel()), v.device)
        call("ssq_round_reg", vp, v.numel(), float(lam), float(b), _vp(loss), None, ws, wsn,
             stream_of(v))
        ctx.save_for_backward(v)
        ctx.cfg = (lam, b)
        return loss[0]

    @staticmethod
    def backward(ctx, g):
        (v,) = ctx.saved_tensors
        lam, b = ctx.cfg
        gv = torch.zeros_like(v)
        tmp = torch.empty(1, dtype=torch.float32, device=v.device)
        ws, wsn = workspace(query("ssq_round_reg_workspace_size", v.numel()), v.device)
        call("ssq_round_reg", _vp(v), v.numel(), float(lam), float(b), _vp(tmp), _vp(gv), ws, wsn,
             stream_of(v))
        return gv * g, None, None


def round_reg(v, lam, b):
    return RoundRegFn.apply(v, lam, b)


def round_reg_value(v, lam, b, out=None):
    """Value only (no autograd), written to a 1-element device tensor."""
    v, vp = fptr(v.detach())
    out = torch.empty(1, dtype=torch.float32, device=v.device) if out is None else out
    ws, wsn = workspace(query("ssq_round_reg_workspace_size", v.numel()), v.device)
    call("ssq_round_reg", vp, v.numel(), float(lam), float(b), _vp(out), None, ws, wsn, stream_of(v))
    return out


# ------------------------------------------------------------------ K10
def inpscale_search(w, delta, raw_zp, n_bits, level, threshold):
    """ChannelQuantMSE.init_scale 'max' (channelQuantMSE.py:203-241) -> inp_scale
    shaped (1, Ci, kh, kw) / (1, Ci)."""
    w, wp = fptr(w.detach())
    d, dp = fptr(delta.detach())
    r, rp = fptr(raw_zp.detach())
    Co = w.shape[0]
    J = w.numel() // Co
    inp = torch.empty((1,) + tuple(w.shape[1:]), dtype=torch.float32, device=w.device)
    call("ssq_inpscale_search", wp, dp, rp, Co, J, n_bits, int(level), float(threshold), _vp(inp),
         stream_of(w))
    return inp


def inpscale_fwd(w, inp, delta, raw_zp, n_bits):
    """ChannelQuantMSE.forward (channelQuantMSE.py:267-276)."""
    w, wp = fptr(w.detach())
    i, ip = fptr(inp.detach())
    d, dp = fptr(delta.detach())
    r, rp = fptr(raw_zp.detach())
    Co = w.shape[0]
    out = torch.empty_like(w)
    call("ssq_inpscale_fwd", wp, ip, dp, rp, Co, w.numel() // Co, n_bits, _vp(out), stream_of(w))
    return out


# ------------------------------------------------------------------ K11 / K14
def _lp_M(pred, reduction):
    if reduction == "none":
        return pred.numel() // pred.shape[1]
    return pred.numel()


class Rows:
    """cache[idx] as a lazy target: the loss pass reads the rows in place
    (ssq_lp_loss_rows) instead of a gathered copy."""

    def __init__(self, cache, idx):
        self.cache, self.idx = cache, idx

    def materialize(self):
        return gather_rows2(self.cache, self.idx)[0]


# ------------------------------------------------------------------ in-place row views
# BRECQ's act phase reads its frozen convs' precomputed outputs and the cached block input
# by the batch indices (quant/block_recon.py ROWS_IN_PLACE).  Instead of gathering each into
# a batch buffer, the buffer is registered as a view of cache[idx] (rows_view) and the K13
# epilogue kernels read the rows in place (ssq_epilogue_*_rows, bit-identical to reading the
# gathered batch).  Any other kernel call reaching the buffer through fptr gathers it first
# (_capi.fptr), as does materialize(); the registry lives for one loop (row_views).
def rows_view(buf, cache, idx):
    """Register buf (a contiguous batch buffer, never read by torch ops while registered) as
    cache[idx]; returns buf."""
    if tuple(buf.shape) != (idx.numel(),) + tuple(cache.shape[1:]) or not buf.is_contiguous() \
            or idx.dtype != torch.int64 or not cache.is_contiguous():
        raise A.SSQError("rows_view: buffer, cache and indices do not match")
    A.ROW_VIEWS[buf.data_ptr()] = (buf, cache, idx)
    return buf


def rows_of(t):
    """(cache, idx) when t is a registered row view, else None."""
    if t is None or not A.ROW_VIEWS:
        return None
    e = A.ROW_VIEWS.get(t.data_ptr())
    return None if e is None or e[0].numel() != t.numel() else (e[1], e[2])


class row_views:
    """Context of a loop that registers row views: the registry and any stage still pending
    (a capture that raised between rows_lazy and the kernel that takes it) are emptied on
    exit, so no later call performs an old loop's copy."""

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        A.ROW_VIEWS.clear()
        A.ROW_STAGE.clear()


def lp_loss_and_grad(pred, tgt, p=2.0, reduction="none", want_grad=True, loss_out=None,
                     relu_mask=False):
    """lp_loss value (1-element device tensor) and d/d pred in one fused pass.  With
    relu_mask, pred is a ReLU output and the gradient is returned at the ReLU's input.
    tgt may be a Rows(cache, idx) target."""
    pred, pp = fptr(pred.detach(), "pred")
    loss = torch.empty(1, dtype=torch.float32, device=pred.device) if loss_out is None else loss_out
    grad = torch.empty_like(pred) if want_grad else None
    ws, wsn = workspace(query("ssq_lp_loss_workspace_size", pred.numel()), pred.device, "loss")
    M = _lp_M(pred, reduction)
    if isinstance(tgt, Rows):
        cache, cp = fptr(tgt.cache.detach(), "tgt cache")
        idx = tgt.idx
        row = cache[0].numel()
        if idx.dtype != torch.int64 or idx.device != pred.device or \
                idx.numel() * row != pred.numel() or tuple(cache.shape[1:]) != tuple(pred.shape[1:]):
            raise A.SSQError("lp_loss: Rows target does not match pred")
        call("ssq_lp_loss_rows", pp, cp, _vp(idx), row, pred.numel(), M, float(p), _vp(loss),
             _vp(grad), None, int(bool(relu_mask)), ws, wsn, stream_of(pred))
        return loss, grad
    tgt, tp = fptr(tgt.detach(), "tgt")
    call("ssq_lp_loss", pp, tp, pred.numel(), M, float(p), _vp(loss),
         _vp(grad), None, int(bool(relu_mask)), ws, wsn, stream_of(pred))
    return loss, grad


class LpLossFn(torch.autograd.Function):
    """lp_loss (quant_layer.py:25-32): forward = value only; backward = one pass that
    writes (1/M)*(p|d|^(p-1))*sgn(d) scaled by the upstream gradient (device scalar)."""

    @staticmethod
    def forward(ctx, pred, tgt, p, reduction):
        loss, _ = lp_loss_and_grad(pred, tgt, p, reduction, want_grad=False)
        ctx.save_for_backward(pred, tgt)
        ctx.cfg = (p, reduction)
        return loss[0]

    @staticmethod
    def backward(ctx, g):
        pred, tgt = ctx.saved_tensors
        p, reduction = ctx.cfg
        pred, tgt = pred.contiguous(), tgt.contiguous()
        grad = torch.empty_like(pred)
        gs = g.detach().reshape(1).to(torch.float32).contiguous()
        call("ssq_lp_loss", _vp(pred), _vp(tgt), pred.numel(), _lp_M(pred, reduction), float(p),
             None, _vp(grad), _vp(gs), 0, None, 0, stream_of(pred))
        return grad, None, None, None


def lp_loss(pred, tgt, p=2.0, reduction="none"):
    return LpLossFn.apply(pred, tgt, float(p), reduction)


def gather_rows2(src0, idx, src1=None, out0=None, out1=None):
    """src[idx] for one or two row-major sources (the cached block input / output)."""
    s0, p0 = fptr(src0, "src0")
    idx = idx.to(device=s0.device, dtype=torch.int64).contiguous()
    n = idx.numel()
    row0 = s0[0].numel()
    d0 = torch.empty((n,) + tuple(s0.shape[1:]), dtype=s0.dtype, device=s0.device) if out0 is None else out0
    if src1 is not None:
        s1, p1 = fptr(src1, "src1")
        row1 = s1[0].numel()
        d1 = torch.empty((n,) + tuple(s1.shape[1:]), dtype=s1.dtype, device=s1.device) if out1 is None else out1
    else:
        s1, p1, row1, d1 = None, None, 0, None
    call("ssq_gather_rows2", p0, _vp(d0), row0, p1, _vp(d1), row1, _vp(idx), n, stream_of(s0))
    return d0, d1


def gather_rows2_staged(src0, slot, n, stage_dst, src1=None, out0=None, out1=None):
    """gather_rows2 with the indices slot[:n] of a device ring row, which the same launch
    also copies whole into stage_dst (ssq_gather_rows2_staged)."""
    s0, p0 = fptr(src0, "src0")
    if slot.dtype != torch.int64 or not slot.is_contiguous() or stage_dst.dtype != torch.int64 \
            or stage_dst.numel() != slot.numel() or slot.device != s0.device:
        raise A.SSQError("gather_rows2_staged: int64 contiguous slot and stage_dst of one size")
    row0 = s0[0].numel()
    d0 = torch.empty((n,) + tuple(s0.shape[1:]), dtype=s0.dtype, device=s0.device) if out0 is None else out0
    if src1 is not None:
        s1, p1 = fptr(src1, "src1")
        row1 = s1[0].numel()
        d1 = torch.empty((n,) + tuple(s1.shape[1:]), dtype=s1.dtype, device=s1.device) if out1 is None else out1
    else:
        s1, p1, row1, d1 = None, None, 0, None
    call("ssq_gather_rows2_staged", p0, _vp(d0), row0, p1, _vp(d1), row1, _vp(slot), n,
         _vp(stage_dst), slot.numel(), stream_of(s0))
    return d0, d1


# ------------------------------------------------------------------ K13 fused epilogue
class BiasActFn(torch.autograd.Function):
    """act((y + bias[c]) + res) in one kernel (conv bias add quant_layer.py:250, residual
    add + ReLU quant_block.py:99-117).  The bias is taken as a constant (no
    reconstruction optimises it); gradients flow to y and res."""

    @staticmethod
    def forward(ctx, y, bias, res, relu):
        y, yp, bp, rp, C, hw, _, (yi, ri), stg = _epilogue_layout(y, bias, res, rows=True,
                                                                 stage=True)
        out = torch.empty_like(y)
        if yi is not None or ri is not None:
            call("ssq_epilogue_fwd_rows", yp, yi, bp, None, None, rp, ri, _vp(out), None,
                 y.numel(), hw, C, int(relu), None, None, 0, 1, *stg, stream_of(y))
        else:
            call("ssq_bias_act", yp, bp, rp, _vp(out), y.numel(), hw, C, int(relu), stream_of(y))
        ctx.relu = int(relu)
        if relu:
            ctx.save_for_backward(out)
        return out

    @staticmethod
    def backward(ctx, g):
        if ctx.relu:
            (out,) = ctx.saved_tensors
            g, gp = fptr(g.contiguous(), "grad")
            gin = torch.empty_like(g)
            call("ssq_relu6_bwd" if ctx.relu == 2 else "ssq_relu_bwd", gp, _vp(out), _vp(gin),
                 g.numel(), stream_of(g))
        else:
            gin = g
        return gin, None, (gin if ctx.needs_input_grad[2] else None), None


class LazyRes:
    """A block's downsample branch whose epilogue is deferred to the block's fused tail: the
    downsample conv's raw output y and its epilogue's inputs (bias, gamma^z / phi^z, no
    activation, no act quantizer).  The tail's pass applies that epilogue itself
    (ssq_epilogue_loss_bwd's res_* arguments) and returns dL/dy; anywhere else the residual is
    materialised with exactly the ops QuantModule.forward runs for it."""

    def __init__(self, y, bias, gamma, phi):
        self.y, self.bias, self.gamma, self.phi = y, bias, gamma, phi

    def materialize(self):
        if self.gamma is not None:
            return epilogue(self.y, self.bias, self.gamma, self.phi, None, 0, None)
        if self.bias is not None:
            return bias_act(self.y, self.bias, None, 0)
        return self.y


def materialize(res):
    """A residual as a tensor with its values: a LazyRes materialised, a row view gathered."""
    if isinstance(res, LazyRes):
        return res.materialize()
    if res is not None and A.ROW_VIEWS:
        A.materialize_rows(res)
    return res


def _unlazy(res):
    """A LazyRes materialised for an epilogue kernel; a row view stays one (the K13 kernels
    read it in place)."""
    return res.materialize() if isinstance(res, LazyRes) else res


# A/B knob: the downsample branch's epilogue deferred into the block's fused tail (LazyRes;
# bit-identical either way)
FOLD_RESIDUAL = os.environ.get("SSQ_FOLD_RESIDUAL", "1") != "0"


# The fused tail also on planes whose rows are not float4 rows (ResNet-18 layer4's 7x7), in
# the kernel's scalar-row form: layer4.1 2114 it/s against 2085 with the three separate
# passes, layer4.0 unchanged (profiles/r3_ab_knobs.txt).  A/B knob: SSQ_TAIL_SCALAR=0.
TAIL_SCALAR = os.environ.get("SSQ_TAIL_SCALAR", "1") != "0"


def _tail_ok(y, res):
    """The fused tail (epilogue_loss_bwd) takes contiguous NCHW float4 rows (hw % 4 == 0,
    16-B aligned), and scalar rows when TAIL_SCALAR is set."""
    if isinstance(res, LazyRes):
        res = res.y
    if not (y.dim() == 4 and y.is_contiguous() and (res is None or res.is_contiguous())):
        return False
    if TAIL_SCALAR:
        return True
    return ((y.shape[2] * y.shape[3]) % 4 == 0 and y.data_ptr() % 16 == 0
            and (res is None or res.data_ptr() % 16 == 0))


def bias_act(y, bias=None, res=None, relu=True, lazy=False):
    """relu: activation code (False/0 identity, True/1 ReLU, 2 ReLU6).  lazy: see
    TAIL_LAZY (the block's final epilogue, fused with the loss and its backward)."""
    if lazy and int(relu) in (0, 1) and _tail_ok(y, res):
        out = torch.empty_like(y)
        out._ssq_tail = (y, bias, None, None, res, int(relu), None)
        return out
    res = _unlazy(res)
    out = BiasActFn.apply(y, bias, res, int(relu))
    if int(relu) == 1:
        # lets a loss that folds the ReLU backward into its own pass (lp_loss relu_mask)
        # back-propagate from the ReLU's inputs directly
        out._ssq_relu_inputs = tuple(t for t in (y, res) if t is not None and t.requires_grad)
    return out


def _epilogue_layout(y, bias, res, rows=False, stage=False):
    """Pointers and (C, hw) of an epilogue's operands.  rows: y / res may stay row views --
    their pointers are then their caches' and the result ends with their row maps' pointers
    (None for an operand that is the batch itself); otherwise a row view is gathered (fptr).
    stage (the K13 forward): a pending stage of the iteration's device words (_capi.ROW_STAGE)
    is taken over by the caller's launch -- the maps then point into the ring row it copies
    from -- and the result ends with (src, dst, n) pointers for ssq_epilogue_fwd_rows, or
    (None, None, 0); without a row map the stage is performed here as a copy."""
    st = None
    if rows and stage:
        st = A.take_row_stage()
    elif A.ROW_STAGE:
        A.flush_row_stage()
    yr = rows_of(y) if rows else None
    rr = rows_of(res) if rows else None
    if yr is not None:
        A.check(y, "conv output")
        yp = _vp(yr[0])
    else:
        y, yp = fptr(y.detach(), "conv output")
    C = y.shape[1] if y.dim() > 1 else 1
    hw = y[0, 0].numel() if y.dim() > 2 else 1
    bp = rp = None
    if bias is not None:
        bias, bp = fptr(bias.detach().reshape(-1), "bias")
        if bias.numel() != C:
            raise A.SSQError("bias_act: bias must have one value per channel")
    if res is not None:
        if rr is not None:
            A.check(res, "residual")
            rp = _vp(rr[0])
        else:
            res, rp = fptr(res.detach(), "residual")
        if res.shape != y.shape:
            raise A.SSQError("bias_act: residual shape mismatch")
    if rows:
        def rmap(t):
            # the static slot's indices are read from the ring row this launch copies
            if st is not None and t.data_ptr() == st[1].data_ptr():
                return _vp(st[0])
            return _vp(t)
        maps = (None if yr is None else rmap(yr[1]), None if rr is None else rmap(rr[1]))
        if st is not None and maps == (None, None):
            st[1].copy_(st[0])
            st = None
        if stage:
            stg = (None, None, 0) if st is None else (_vp(st[0]), _vp(st[1]), st[0].numel())
            return y, yp, bp, rp, C, hw, (bias, res), maps, stg
        return y, yp, bp, rp, C, hw, (bias, res), maps
    return y, yp, bp, rp, C, hw, (bias, res)


class BiasActQuantFn(torch.autograd.Function):
    """K13 epilogue followed by the per-tensor activation fake-quant, one pass:
    fq(act((y + bias[c]) + res)) (quant_layer.py:250,270-272; quant_block.py:99-118).
    The pre-quant activation is written only when a backward will need it.  Backward:
    the STE / delta / zero-point gradients of FakeQuantFn with the ReLU backward folded
    into the same pass (ssq_fq_relu_bwd)."""

    @staticmethod
    def forward(ctx, y, bias, res, delta, zp, relu, n_bits, sym, keep):
        y, yp, bp, rp, C_, hw, hold, (yi, ri), stg = _epilogue_layout(y, bias, res, rows=True,
                                                                     stage=True)
        d, dp = fptr(delta.detach().reshape(-1), "delta")
        z, zpp = fptr(zp.detach().reshape(-1), "zero_point")
        if d.numel() != 1 or z.numel() != 1:
            raise A.SSQError("bias_act_fq: per-tensor activation quantizer only")
        lo, hi = qrange(n_bits, sym)
        out = torch.empty_like(y) if keep else None
        yq = torch.empty_like(y)
        if yi is not None or ri is not None:
            call("ssq_epilogue_fwd_rows", yp, yi, bp, None, None, rp, ri, _vp(out), _vp(yq),
                 y.numel(), hw, C_, int(relu), dp, zpp, lo, hi, *stg, stream_of(y))
        else:
            call("ssq_bias_act_fq", yp, bp, rp, _vp(out), _vp(yq), y.numel(), hw, C_, int(relu),
                 dp, zpp, lo, hi, stream_of(y))
        ctx.relu, ctx.q = int(relu), (lo, hi)
        if keep:
            ctx.save_for_backward(out, delta, zp)
        return yq

    @staticmethod
    def backward(ctx, g):
        out, delta, zp = ctx.saved_tensors
        lo, hi = ctx.q
        g, gp = fptr(g.contiguous(), "grad")
        d, z = delta.detach().contiguous(), zp.detach().contiguous()
        need_in = ctx.needs_input_grad[0] or ctx.needs_input_grad[2]
        gin = torch.empty_like(g) if need_in else None
        gd = torch.empty(1, dtype=torch.float32, device=g.device) if ctx.needs_input_grad[3] else None
        gz = torch.empty(1, dtype=torch.float32, device=g.device) if ctx.needs_input_grad[4] else None
        n = g.numel()
        ws, wsn = workspace(query("ssq_fq_bwd_workspace_size", n, n, 1), g.device)
        if ctx.relu:
            call("ssq_fq_relu6_bwd" if ctx.relu == 2 else "ssq_fq_relu_bwd", _vp(out), gp, _vp(d), _vp(z), n, lo, hi, _vp(gin), _vp(gd),
                 _vp(gz), ws, wsn, stream_of(g))
        else:
            call("ssq_fq_bwd", _vp(out), gp, _vp(d), _vp(z), n, n, 1, lo, hi, _vp(gin), _vp(gd),
                 _vp(gz), ws, wsn, stream_of(g))
        return (gin if ctx.needs_input_grad[0] else None, None,
                gin if ctx.needs_input_grad[2] else None,
                None if gd is None else gd.view(delta.shape),
                None if gz is None else gz.view(zp.shape), None, None, None, None)


def bias_act_quant(y, bias, res, relu, delta, zp, n_bits, sym=False):
    """bias_act followed by fake_quant(delta, zp) in one pass (per-tensor quantizer)."""
    res = _unlazy(res)
    keep = torch.is_grad_enabled() and any(
        t is not None and t.requires_grad for t in (y, res, delta, zp))
    return BiasActQuantFn.apply(y, bias, res, delta, zp, int(relu), n_bits, sym, keep)


class EpilogueFn(torch.autograd.Function):
    """act(((y + bias[c]) * gamma[c] + phi[c]) (+ res)) [-> per-tensor act fake-quant] in one
    pass (quant_layer.py:250,266-272; quant_block.py:99-118) -- the general K13 epilogue,
    with the --bias_cal affine gamma^z/phi^z.  Backward (ssq_epilogue_bwd) recomputes the
    pre-activation from the conv output y and returns the y / res / gamma / phi / delta /
    zero_point gradients of the reference's op sequence."""

    @staticmethod
    def forward(ctx, y, bias, gamma, phi, res, delta, zp, relu, n_bits, sym):
        y, yp, bp, rp, C_, hw, _, (yi, ri), stg = _epilogue_layout(y, bias, res, rows=True,
                                                                  stage=True)
        gm, gmp = fptr(gamma.detach().reshape(-1), "gamma") if gamma is not None else (None, None)
        ph, php = fptr(phi.detach().reshape(-1), "phi") if phi is not None else (None, None)
        if gm is not None and (gm.numel() != C_ or ph.numel() != C_):
            raise A.SSQError("epilogue: gamma / phi must have one value per channel")
        quant = delta is not None
        if quant:
            d, dp = fptr(delta.detach().reshape(-1), "delta")
            z, zpp = fptr(zp.detach().reshape(-1), "zero_point")
            if d.numel() != 1 or z.numel() != 1:
                raise A.SSQError("epilogue: per-tensor activation quantizer only")
            lo, hi = qrange(n_bits, sym)
        else:
            dp = zpp = None
            lo, hi = 0, 1
        out = torch.empty_like(y)
        if yi is not None or ri is not None:
            call("ssq_epilogue_fwd_rows", yp, yi, bp, gmp, php, rp, ri, None if quant else _vp(out),
                 _vp(out) if quant else None, y.numel(), hw, C_, int(relu), dp, zpp, lo, hi,
                 *stg, stream_of(y))
        else:
            call("ssq_epilogue_fwd", yp, bp, gmp, php, rp, None if quant else _vp(out),
                 _vp(out) if quant else None, y.numel(), hw, C_, int(relu), dp, zpp, lo, hi,
                 stream_of(y))
        ctx.cfg = (int(relu), lo, hi, quant, C_, hw)
        ctx.save_for_backward(y, bias, gamma, phi, res, delta, zp)
        return out

    @staticmethod
    def backward(ctx, g):
        y, bias, gamma, phi, res, delta, zp = ctx.saved_tensors
        relu, lo, hi, quant, C_, hw = ctx.cfg
        return _epilogue_backward(g, y, bias, gamma, phi, res, delta, zp, relu, lo, hi, quant,
                                  C_, hw, ctx.needs_input_grad)


def _epilogue_backward(g, y, bias, gamma, phi, res, delta, zp, relu, lo, hi, quant, C_, hw, need):
    """ssq_epilogue_bwd for EpilogueFn (need = its needs_input_grad) and EpiConvGemmFn:
    EpilogueFn.backward's return tuple."""
    g, gp = fptr(g.contiguous(), "grad")
    dev_ = g.device

    def flat(t):
        return None if t is None else t.detach().reshape(-1).contiguous()
    b, gm, ph, r = flat(bias), flat(gamma), flat(phi), res
    d, z = flat(delta), flat(zp)
    yr, rr = rows_of(y), rows_of(r)
    gy = torch.empty_like(g) if need[0] else None
    gres = torch.empty_like(g) if (res is not None and need[4]) else None
    ggm, gm_into = _grad_dest(gamma, C_, dev_, need[2])
    gph, ph_into = _grad_dest(phi, C_, dev_, need[3])
    gd = torch.empty(1, device=dev_) if (quant and need[5]) else None
    gz = torch.empty(1, device=dev_) if (quant and need[6]) else None
    N = g.numel() // (C_ * hw)
    # two alternating slots: a queued finalize of the previous call still reads its own
    ws, wsn = workspace(query("ssq_epilogue_bwd_workspace_size", N * C_), dev_, _epi_slot())
    if yr is not None or rr is not None:
        call("ssq_epilogue_bwd_rows", gp, _vp(y if yr is None else yr[0]),
             None if yr is None else _vp(yr[1]), _vp(b), _vp(gm), _vp(ph),
             _vp(r.contiguous() if (r is not None and rr is None) else (rr[0] if rr else None)),
             None if rr is None else _vp(rr[1]), N, C_, hw, int(relu), _vp(d), _vp(z), lo, hi,
             _vp(gy), _vp(gres), _vp(ggm), _vp(gph), _vp(gd), _vp(gz), ws, wsn, stream_of(g))
    else:
        call("ssq_epilogue_bwd", gp, _vp(y), _vp(b), _vp(gm), _vp(ph),
             _vp(r.contiguous() if r is not None else None), N, C_, hw, int(relu), _vp(d),
             _vp(z), lo, hi, _vp(gy), _vp(gres), _vp(ggm), _vp(gph), _vp(gd), _vp(gz), ws, wsn,
             stream_of(g))
    shape = (lambda t, o: None if o is None else o.view(t.shape))
    return (gy if need[0] else None, None, None if gm_into else shape(gamma, ggm),
            None if ph_into else shape(phi, gph), gres, shape(delta, gd), shape(zp, gz), None,
            None, None)


_EPI_SLOT = [0]


def _epi_slot():
    _EPI_SLOT[0] ^= 1
    return _epi_slot_name()


def _epi_slot_name():
    """The workspace slot of the last epilogue backward (tests read its row records)."""
    return "epi%d" % _EPI_SLOT[0]


def set_deferred_finalize(on):
    """Queue the loss / epilogue-backward finalizes onto the next host launch (include/ssq.h,
    csrc/fin_tasks.h); returns the previous setting."""
    return bool(query("ssq_set_deferred_finalize", int(bool(on))))


def flush_finalize(device=None):
    """Launch the finalizes still queued on the current stream."""
    dev_ = torch.device("cuda", torch.cuda.current_device()) if device is None else device
    call("ssq_flush_finalize", C.c_void_p(torch.cuda.current_stream(dev_).cuda_stream))


class deferred_finalize:
    """Context: deferral on inside, flushed and restored on exit (the recon loop body)."""

    def __init__(self, on=True, device=None):
        self.on, self.device = on, device

    def __enter__(self):
        self.prev = set_deferred_finalize(self.on) if self.on else None
        return self

    def __exit__(self, *exc):
        if self.on:
            try:
                flush_finalize(self.device)
            finally:
                set_deferred_finalize(self.prev)


class deferred_prep_fwd:
    """Context (the fused loop's iteration start): the prepared adaShift forward launched
    inside it rides on the next batch gather of its stream (include/ssq.h,
    csrc/prep_ride.h); a forward still queued at exit is launched then."""

    def __init__(self, on=True, device=None):
        self.on, self.device = on, device

    def __enter__(self):
        self.prev = bool(query("ssq_set_deferred_prep_fwd", 1)) if self.on else None
        return self

    def __exit__(self, *exc):
        if self.on:
            dev_ = torch.device("cuda", torch.cuda.current_device()) if self.device is None \
                else self.device
            try:
                call("ssq_flush_prep_fwd", C.c_void_p(torch.cuda.current_stream(dev_).cuda_stream))
            finally:
                query("ssq_set_deferred_prep_fwd", int(self.prev))


# Set by the fused recon loop around its block forward to the block it reconstructs: that
# block's final epilogue is not run; its output is returned as a placeholder carrying the
# epilogue's inputs (_ssq_tail), and the loop runs forward + loss + backward of that
# epilogue in one pass (epilogue_loss_bwd).  Only consumed by BaseQuantBlock._tail, and
# only by the block identical to TAIL_LAZY[0] (nested blocks and hooked blocks run eagerly).
TAIL_LAZY = [None]


# ------------------------------------------------------------------ K13 epilogue into an im2col GEMM
# A ResNet BasicBlock's conv1 epilogue feeds only conv2.  Where conv2's forward and weight
# gradient run as GEMMs over one im2col matrix (ResNet-18 layer3 / layer4: _use_fwd_gemm),
# the block marks conv2 as the consumer (EPI_CONSUMER) while conv1 runs; conv1 then returns
# a placeholder carrying its raw output and its epilogue's inputs (LazyEpi), and conv2 builds
# its im2col matrix from them with the epilogue applied on the fly (ssq_gemm_col_epilogue):
# the epilogue's forward launch and its activation-sized output are gone, the bits are the
# same (col is the im2col of the same values; the backward runs the same ssq_epilogue_bwd on
# the same input gradient).  Any other consumer materialises the placeholder with exactly
# the ops QuantModule.forward runs.  Off by default (SSQ_EPI_GEMM=1 turns it on): the im2col
# build evaluates the epilogue once per column entry, R*S = 9 times per activation, and that
# costs more than the launch it saves -- bench.py's recon loops, ABAB on one box (r5j,
# profiles/r5_epi_gemm_ab.txt): layer3.0 1980 vs 2001 it/s, layer3.1 2012 vs 2029, layer4.0
# 2341 vs 2344, layer4.1 2196 vs 2215 with the fold on vs off.
EPI_INTO_GEMM = os.environ.get("SSQ_EPI_GEMM", "0") == "1"
EPI_CONSUMER = [None]


class LazyEpi:
    """conv1's raw output y and its K13 epilogue's inputs (QuantModule.forward's fused
    branch: bias, gamma^z / phi^z, activation code, per-tensor act quantizer)."""

    def __init__(self, y, bias, gamma, phi, relu, q):
        self.y, self.bias, self.gamma, self.phi, self.relu, self.q = y, bias, gamma, phi, relu, q

    def materialize(self):
        y, bias, gamma, phi, relu, q = self.y, self.bias, self.gamma, self.phi, self.relu, self.q
        if gamma is not None:
            return epilogue(y, bias, gamma, phi, None, relu, q)
        if q is not None:
            return bias_act_quant(y, bias, None, relu, q.delta, q.zero_point, q.n_bits, q.sym)
        if bias is not None or relu:
            return bias_act(y, bias, None, relu)
        return y


def lazy_epilogue(y, bias, gamma, phi, relu, q):
    out = torch.empty_like(y)
    out._ssq_epi = LazyEpi(y, bias, gamma, phi, int(relu), q)
    return out


def materialize_epi(x):
    epi = getattr(x, "_ssq_epi", None)
    return x if epi is None else epi.materialize()


class EpiConvGemmFn(torch.autograd.Function):
    """conv2d(epilogue(y), W) (no bias, ungrouped, dilation 1) as ONE im2col build with the
    epilogue folded in (ssq_gemm_col_epilogue) + the strided-batched GEMM of conv_fwd_gemm.
    Backward: the input gradient on MIOpen (the input's values are not read), the weight
    gradient as conv_wgrad_gemm over the saved im2col matrix, then the epilogue's backward
    (ssq_epilogue_bwd) on that input gradient -- the unfused path's kernels and operands."""

    @staticmethod
    def forward(ctx, y, bias, gamma, phi, delta, zp, weight, cfg):
        relu, n_bits, sym, stride, padding = cfg
        Nb, C_, H, W, Co, R, S, st, pad, OH, OW = _gemm_geo(y.shape, weight.shape, stride, padding)
        y, yp = fptr(y.detach(), "conv output")
        flat = (lambda t, nm: (None, None) if t is None else fptr(t.detach().reshape(-1), nm))
        b, bp = flat(bias, "bias")
        gm, gmp = flat(gamma, "gamma")
        ph, php = flat(phi, "phi")
        d, dp = flat(delta, "delta")
        z, zpp = flat(zp, "zero_point")
        for t, nm in ((b, "bias"), (gm, "gamma"), (ph, "phi")):
            if t is not None and t.numel() != C_:
                raise A.SSQError(f"epilogue into GEMM: {nm} must have one value per channel")
        quant = d is not None
        lo, hi = qrange(n_bits, sym) if quant else (0, 1)
        NP, CRS = Nb * OH * OW, C_ * R * S
        col = torch.empty(NP, CRS, dtype=torch.float32, device=y.device)
        call("ssq_gemm_col_epilogue", yp, bp, gmp, php, int(relu), dp, zpp, lo, hi, Nb, C_, H, W,
             R, S, st, pad, _vp(col), stream_of(y))
        out = torch.matmul(weight.detach().reshape(Co, CRS), col.view(Nb, OH * OW, CRS).transpose(1, 2))
        ctx.save_for_backward(y, bias, gamma, phi, delta, zp, weight, col)
        ctx.cfg = (int(relu), lo, hi, quant, C_, H * W, stride, padding)
        return out.view(Nb, Co, OH, OW)

    @staticmethod
    def backward(ctx, g):
        y, bias, gamma, phi, delta, zp, weight, col = ctx.saved_tensors
        relu, lo, hi, quant, C_, hw, stride, padding = ctx.cfg
        need = ctx.needs_input_grad
        g = g.contiguous()
        # the conv's input: only its shape matters to the input gradient and the dy operand
        x_like = torch.empty(y.shape, dtype=y.dtype, device=y.device)
        gw = None
        if need[6]:
            _, dy2 = gemm_operands(x_like, g, weight.shape, stride, padding, want_col=False,
                                   want_dy2=True)
            gw = torch.matmul(dy2, col).view(tuple(weight.shape))
        if not any(need[:6]):
            return None, None, None, None, None, None, gw, None
        gx = torch.ops.aten.convolution_backward(
            g, x_like, weight, None, _pair(stride), _pair(padding), [1, 1], False, [0, 0], 1,
            (True, False, False))[0]
        gy, _, ggm, gph, _, gd, gz, _, _, _ = _epilogue_backward(
            gx, y, bias, gamma, phi, None, delta, zp, relu, lo, hi, quant, C_, hw,
            (need[0], False, need[2], need[3], False, need[4], need[5]))
        return gy, None, ggm, gph, gd, gz, gw, None


def epi_conv_gemm(x, weight, stride, padding):
    """conv2d of a LazyEpi placeholder x through EpiConvGemmFn."""
    e = x._ssq_epi
    q = e.q
    cfg = (e.relu, q.n_bits if q is not None else 8, q.sym if q is not None else False,
           stride, padding)
    return EpiConvGemmFn.apply(e.y, e.bias, e.gamma, e.phi, None if q is None else q.delta,
                               None if q is None else q.zero_point, weight, cfg)


def epilogue(y, bias, gamma, phi, res, relu, q=None, lazy=False):
    """EpilogueFn with q an (initialised, per-tensor) act quantizer or None.  lazy: see
    TAIL_LAZY (the placeholder must only reach epilogue_loss_bwd)."""
    if lazy and int(relu) in (0, 1) and _tail_ok(y, res):
        out = torch.empty_like(y)
        out._ssq_tail = (y, bias, gamma, phi, res, int(relu), q)
        return out
    res = _unlazy(res)
    if q is None:
        return EpilogueFn.apply(y, bias, gamma, phi, res, None, None, int(relu), 8, False)
    return EpilogueFn.apply(y, bias, gamma, phi, res, q.delta, q.zero_point, int(relu), q.n_bits,
                            q.sym)


def epilogue_loss_bwd(tail, tgt, M, p=2.0):
    """The fused tail (ssq_epilogue_loss_bwd): for a lazy epilogue placeholder's inputs and a
    Rows target, the lp_loss value at power p (1-element device tensor, mean over M) and the
    gradients the epilogue's backward returns -- (loss, gy, gres, ggamma, gphi, gdelta, gzp,
    gres_gamma, gres_phi), None where the input needs none -- bit-identical to epilogue ->
    lp_loss_and_grad -> backward.  A LazyRes residual (the downsample's deferred epilogue) is
    applied in the same pass: gres is then dL/d(its raw conv output) and gres_gamma /
    gres_phi its gamma^z / phi^z gradients."""
    y, bias, gamma, phi, res, relu, q = tail
    if not isinstance(tgt, Rows):
        raise A.SSQError("epilogue_loss_bwd: the target must be a Rows view of the cache")
    lres = res if isinstance(res, LazyRes) else None
    if lres is not None:
        res = lres.y
    y, yp, bp, rp, C_, hw, _, (yi, ri) = _epilogue_layout(y, bias, res, rows=True)
    dev_ = y.device
    cache, cp = fptr(tgt.cache.detach(), "tgt cache")
    idx = tgt.idx
    N = y.shape[0]
    if idx.dtype != torch.int64 or idx.numel() != N or tuple(cache.shape[1:]) != tuple(y.shape[1:]):
        raise A.SSQError("epilogue_loss_bwd: Rows target does not match the output")
    flat = (lambda t: None if t is None else t.detach().reshape(-1).contiguous())
    gm, ph = flat(gamma), flat(phi)
    if q is not None:
        d, z = flat(q.delta), flat(q.zero_point)
        lo, hi = qrange(q.n_bits, q.sym)
    else:
        d = z = None
        lo, hi = 0, 1
    loss = torch.empty(1, dtype=torch.float32, device=dev_)
    gy = torch.empty_like(y)
    gres = torch.empty_like(y) if (res is not None and res.requires_grad) else None
    ggm, gm_into = _grad_dest(gamma, C_, dev_, gamma is not None and gamma.requires_grad)
    gph, ph_into = _grad_dest(phi, C_, dev_, phi is not None and phi.requires_grad)
    rbp = rgp = rphp = None
    grg, grph, rg_into, rph_into = None, None, False, False
    if lres is not None:
        if lres.bias is not None:
            rb, rbp = fptr(lres.bias.detach().reshape(-1), "residual bias")
            if rb.numel() != C_:
                raise A.SSQError("epilogue_loss_bwd: residual bias must have one value per channel")
        if lres.gamma is not None:
            rg, rgp = fptr(lres.gamma.detach().reshape(-1), "residual gamma")
            rph_, rphp = fptr(lres.phi.detach().reshape(-1), "residual phi")
            if rg.numel() != C_ or rph_.numel() != C_:
                raise A.SSQError("epilogue_loss_bwd: residual gamma / phi must have one value per channel")
            grg, rg_into = _grad_dest(lres.gamma, C_, dev_, lres.gamma.requires_grad)
            grph, rph_into = _grad_dest(lres.phi, C_, dev_, lres.phi.requires_grad)
    gd = torch.empty(1, device=dev_) if (q is not None and q.delta.requires_grad) else None
    gz = torch.empty(1, device=dev_) if (q is not None and q.zero_point.requires_grad) else None
    ws, wsn = workspace(query("ssq_epilogue_bwd_workspace_size", N * C_), dev_, _epi_slot())
    if yi is not None or ri is not None:
        call("ssq_epilogue_loss_bwd_rows", cp, _vp(idx), int(M), float(p), _vp(loss), yp, yi, bp,
             _vp(gm), _vp(ph), rp, ri, rbp, rgp, rphp, N, C_, hw, int(relu), _vp(d), _vp(z), lo,
             hi, _vp(gy), _vp(gres), _vp(ggm), _vp(gph), _vp(grg), _vp(grph), _vp(gd), _vp(gz),
             ws, wsn, stream_of(y))
    else:
        call("ssq_epilogue_loss_bwd", cp, _vp(idx), int(M), float(p), _vp(loss), yp, bp, _vp(gm),
             _vp(ph), rp, rbp, rgp, rphp, N, C_, hw, int(relu), _vp(d), _vp(z), lo, hi, _vp(gy),
             _vp(gres), _vp(ggm), _vp(gph), _vp(grg), _vp(grph), _vp(gd), _vp(gz), ws, wsn,
             stream_of(y))
    # a gradient written into its GRAD_INTO slice is not handed back (already in place)
    return (loss, gy, gres, None if gm_into else ggm, None if ph_into else gph, gd, gz,
            None if rg_into else grg, None if rph_into else grph)


def adam_step(params, grads, exp_avgs, exp_avg_sqs, beta1, beta2, eps, hyper=None,
              neg_step_size=0.0, bc2_sqrt=1.0):
    """One torch.optim.Adam (single-tensor form) step for every tensor, one launch.
    hyper: device [neg_step_size, bias_correction2_sqrt] (graph-capturable) or None."""
    n = len(params)
    P = C.c_void_p * n
    pa, ga, ma, va = P(), P(), P(), P()
    na = (C.c_int64 * n)()
    for k, (p_, g_, m_, v_) in enumerate(zip(params, grads, exp_avgs, exp_avg_sqs)):
        for t, nm in ((p_, "param"), (g_, "grad"), (m_, "exp_avg"), (v_, "exp_avg_sq")):
            A.check(t, nm)
            if not t.is_contiguous():
                raise A.SSQError(f"adam_step: {nm} must be contiguous")
        pa[k], ga[k], ma[k], va[k] = p_.data_ptr(), g_.data_ptr(), m_.data_ptr(), v_.data_ptr()
        na[k] = p_.numel()
    call("ssq_adam", n, pa, ga, ma, va, na, float(1 - beta1), float(beta2), float(1 - beta2),
         float(eps), _vp(hyper), float(neg_step_size), float(bc2_sqrt), stream_of(params[0]))


def fc_recon_iter(x_cache, tgt_cache, slot, bs, w, v, what, delta, zp, n_bits, bias, exp_avg,
                  exp_avg_sq, beta1, beta2, eps, g=None, gv_out=None, loss_out=None):
    """One fused BRECQ AdaRound iteration of a Linear layer (ssq_fc_recon_iter, K19): the
    forward on what = AdaRound(w, v) (the first call's from adaround(), every later one's
    written by the previous call), the p = 2 loss and its gradient, then dW, V's gradient
    with the rounding regulariser, V's Adam step and the next what, in two launches.  slot:
    int64 device words (bs indices, then (lambda, b, -lr/bc1, sqrt(bc2)) as fp32).
    Returns (loss, g)."""
    xc, xp = fptr(x_cache, "x cache")
    tc, tp = fptr(tgt_cache, "target cache")
    Co, Ci = int(w.shape[0]), int(w.shape[1])
    if xc.shape[1:].numel() != Ci or tc.shape[1:].numel() != Co or slot.dtype != torch.int64 \
            or not slot.is_contiguous() or slot.numel() < bs + 2:
        raise A.SSQError("fc_recon_iter: shapes / slot")
    for t, nm in ((w, "weight"), (v, "V"), (what, "W^"), (exp_avg, "exp_avg"),
                  (exp_avg_sq, "exp_avg_sq")):
        A.check(t, nm)
        if not t.is_contiguous() or t.numel() != Co * Ci:
            raise A.SSQError(f"fc_recon_iter: {nm} must be contiguous [Co, Ci]")
    d, dp = fptr(delta.detach().reshape(-1), "delta")
    z, zpp = fptr(zp.detach().reshape(-1), "zero_point")
    bt, bp = fptr(bias.detach().reshape(-1), "bias") if bias is not None else (None, None)
    dev_ = w.device
    g = torch.empty(bs, Co, device=dev_) if g is None else g
    loss = torch.empty(1, device=dev_) if loss_out is None else loss_out
    ws, wsn = workspace(query("ssq_fc_recon_workspace_size", Co, Ci, bs), dev_, "fc")
    call("ssq_fc_recon_iter", xp, tp, _vp(slot), bs, _vp(w), _vp(v), _vp(what), dp, zpp, 0,
         2 ** n_bits - 1, bp, Co, Ci, float(1 - beta1), float(beta2), float(1 - beta2),
         float(eps), _vp(exp_avg), _vp(exp_avg_sq), _vp(g), _vp(gv_out), _vp(loss), ws, wsn,
         stream_of(w))
    return loss, g


def adam_arm(params, exp_avgs, exp_avg_sqs, beta1, beta2, eps, hyper):
    """Arm one Adam step of `params` (include/ssq.h ssq_adam_arm): the next prepared alpha
    backward on the current stream applies it where the gradients are finalised, when it
    can take all of it.  adam_take() then says whether it did."""
    n = len(params)
    P = C.c_void_p * n
    pa, ma, va = P(), P(), P()
    na = (C.c_int64 * n)()
    for k, (p_, m_, v_) in enumerate(zip(params, exp_avgs, exp_avg_sqs)):
        for t, nm in ((p_, "param"), (m_, "exp_avg"), (v_, "exp_avg_sq")):
            A.check(t, nm)
            if not t.is_contiguous():
                raise A.SSQError(f"adam_arm: {nm} must be contiguous")
        pa[k], ma[k], va[k] = p_.data_ptr(), m_.data_ptr(), v_.data_ptr()
        na[k] = p_.numel()
    call("ssq_adam_arm", n, pa, ma, va, na, float(1 - beta1), float(beta2), float(1 - beta2),
         float(eps), _vp(hyper), stream_of(params[0]))


def adam_take(device=None):
    """True when the armed Adam step ran inside a launch; disarms either way."""
    dev_ = torch.device("cuda", torch.cuda.current_device()) if device is None else device
    return bool(query("ssq_adam_take", C.c_void_p(torch.cuda.current_stream(dev_).cuda_stream)))


def stream_copy(src, dst):
    call("ssq_stream_copy", _vp(src), _vp(dst), src.numel(), stream_of(src))


def stream_read(src, sink):
    """HBM read-only probe over src (K1 geometry); sink is never written in practice."""
    call("ssq_stream_probe", _vp(src), _vp(sink), src.numel(), 1, stream_of(src))


def stream_write(dst):
    """HBM write-only probe over dst (K1 geometry)."""
    call("ssq_stream_probe", None, _vp(dst), dst.numel(), 2, stream_of(dst))


def set_variant(v):
    return query("ssq_set_variant", int(v))


# ------------------------------------------------------------------ K15/K16 packed export
def pack_encode(what, zp, d1, per_ci, d2, n_bits, qmin, qmax):
    """Hard W_hat -> (packed codes as a uint8 tensor, number of elements whose decode is not
    bit-identical; 0 = exact).  W_hat = ((q - zp[co]) * d1) (* d2[j])."""
    w, wp = fptr(what.detach(), "W_hat")
    Co, Ci, Kk, _ = geometry(w)
    z, zpp = fptr(zp.detach().reshape(-1), "zero_point")
    a, ap = fptr(d1.detach().reshape(-1), "scale")
    b, bp = fptr(d2.detach().reshape(-1), "col_scale") if d2 is not None else (None, None)
    if z.numel() != Co or a.numel() != (Co * Ci if per_ci else Co) or \
            (b is not None and b.numel() != Ci * Kk):
        raise A.SSQError("pack_encode: zp / scale / col_scale sizes do not match the weight")
    nbytes = query("ssq_pack_bytes", w.numel(), n_bits)
    packed = torch.empty(max(nbytes, 1), dtype=torch.uint8, device=w.device)[:nbytes]
    bad = torch.zeros(1, dtype=torch.int32, device=w.device)
    call("ssq_pack_encode", wp, zpp, ap, int(per_ci), bp, Co, Ci, Kk, n_bits, qmin, qmax,
         _vp(packed), _vp(bad), stream_of(w))
    return packed, int(bad.item())


def pack_decode(packed, shape, zp, d1, per_ci, d2, n_bits, qmin):
    """Packed codes -> W_hat (fp32, `shape`)."""
    if packed.device.type != "cuda" or packed.dtype != torch.uint8:
        raise A.SSQError("pack_decode: packed codes must be a uint8 tensor on the HIP device")
    out = torch.empty(shape, dtype=torch.float32, device=packed.device)
    Co, Ci, Kk, _ = geometry(out)
    if packed.numel() < query("ssq_pack_bytes", out.numel(), n_bits):
        raise A.SSQError("pack_decode: packed buffer too small for the shape")
    packed = packed.contiguous()
    z, zpp = fptr(zp.reshape(-1), "zero_point")
    a, ap = fptr(d1.reshape(-1), "scale")
    b, bp = fptr(d2.reshape(-1), "col_scale") if d2 is not None else (None, None)
    call("ssq_pack_decode", _vp(packed), zpp, ap, int(per_ci), bp, Co, Ci, Kk, n_bits, qmin,
         _vp(out), stream_of(out))
    return out


# ------------------------------------------------------------------ K17 conv weight gradient
def conv_wgrad_supported(x, weight, stride, padding, dilation, groups):
    """Shapes ssq_conv_wgrad handles: 4-D fp32 NCHW on the device, square stride /
    padding, dilation 1, and a plan whose LDS tile fits (nonzero workspace size)."""
    if x.dim() != 4 or weight.dim() != 4 or not x.is_cuda or x.dtype != torch.float32:
        return False
    st = stride if isinstance(stride, int) else stride[0]
    pad = padding if isinstance(padding, int) else padding[0]
    if not isinstance(stride, int) and len(set(stride)) != 1:
        return False
    if not isinstance(padding, int) and (isinstance(padding, str) or len(set(padding)) != 1):
        return False
    if (dilation if isinstance(dilation, int) else max(dilation)) != 1:
        return False
    Nb, C, H, W = (int(v) for v in x.shape)
    Co, _, R, S = (int(v) for v in weight.shape)
    return query("ssq_conv_wgrad_workspace_size", Nb, C, H, W, Co, R, S, int(st), int(pad),
                 int(groups)) > 0


def wgrad_kind(x_shape, w_shape, stride, padding, groups):
    """The K17 kernel ssq_conv_wgrad runs for this shape (0 unsupported, 1 row tile,
    2 im2col-DMA, 3 band with 16-B staging, 4 1x1 GEMM, 5 depthwise, 6 band with 4-B
    staging)."""
    st = stride if isinstance(stride, int) else stride[0]
    pad = padding if isinstance(padding, int) else padding[0]
    Nb, C, H, W = (int(v) for v in x_shape)
    Co, _, R, S = (int(v) for v in w_shape)
    return int(query("ssq_conv_wgrad_kind", Nb, C, H, W, Co, R, S, int(st), int(pad),
                     int(groups)))


def set_wgrad_form(form):
    """K17 non-depthwise form: 0 auto, 1 input-row-tile (+1x1 GEMM), 2 im2col-DMA, 3 band
    (3x3 pad 1 shapes, Cin / Cout multiples of 32, else the row tile), 4 band at 4 waves per
    workgroup (one per SIMD; 3 runs 8); returns the previous value."""
    return int(query("ssq_conv_wgrad_set_form", int(form)))


def conv_wgrad(x, dy, w_shape, stride, padding, groups):
    """d loss / d weight of F.conv2d(x, w, stride, padding, groups) given dy (K17)."""
    st = stride if isinstance(stride, int) else stride[0]
    pad = padding if isinstance(padding, int) else padding[0]
    x, xp = fptr(x.detach(), "x")
    dy, dp = fptr(dy.detach(), "dy")
    Nb, C, H, W = (int(v) for v in x.shape)
    Co, _, R, S = (int(v) for v in w_shape)
    dims = (Nb, C, H, W, Co, R, S, int(st), int(pad), int(groups))
    ws, wsn = workspace(query("ssq_conv_wgrad_workspace_size", *dims), x.device)
    dw = torch.empty(tuple(w_shape), dtype=torch.float32, device=x.device)
    call("ssq_conv_wgrad", xp, dp, *dims, _vp(dw), ws, wsn, stream_of(x))
    return dw


def _gemm_geo(x_shape, w_shape, stride, padding):
    st = stride if isinstance(stride, int) else stride[0]
    pad = padding if isinstance(padding, int) else padding[0]
    Nb, C_, H, W = (int(v) for v in x_shape)
    Co, _, R, S = (int(v) for v in w_shape)
    OH, OW = (H + 2 * pad - R) // st + 1, (W + 2 * pad - S) // st + 1
    return Nb, C_, H, W, Co, R, S, int(st), int(pad), OH, OW


def gemm_operands(x, dy, w_shape, stride, padding, want_col=True, want_dy2=True):
    """ssq_wgrad_gemm_operands: the im2col matrix col (N*P x C*R*S) of x and/or the
    permuted gradient dy2 (Co x N*P), in one launch."""
    shape = x.shape if x is not None else None
    Nb, C_, H, W, Co, R, S, st, pad, OH, OW = _gemm_geo(shape, w_shape, stride, padding)
    NP = Nb * OH * OW
    dev_ = (x if x is not None else dy).device
    col = torch.empty(NP, C_ * R * S, dtype=torch.float32, device=dev_) if want_col else None
    dy2 = torch.empty(Co, NP, dtype=torch.float32, device=dev_) if want_dy2 else None
    # (the contiguous tensors are held to the launch: a copy made here must not be freed
    # and its block reused by the next one before the kernel has read it)
    xt, xp = fptr(x.detach(), "x") if want_col else (None, None)
    dt, dp = fptr(dy.detach(), "dy") if want_dy2 else (None, None)
    call("ssq_wgrad_gemm_operands", xp, dp, Nb, C_, H, W, Co, R, S, st, pad, _vp(col), _vp(dy2),
         stream_of(col if want_col else dy2))
    return col, dy2


def conv_wgrad_gemm(x, dy, w_shape, stride, padding, col=None):
    """The conv weight gradient as ONE fp32 library GEMM: dw = dy2 @ col
    (torch.matmul -> hipBLASLt; one kernel per shape, bit-identical run to run), the
    operands from ssq_wgrad_gemm_operands (col may be the forward's, saved).  Ungrouped
    convs.  Faster than the band kernel on small output planes."""
    c2, dy2 = gemm_operands(x if col is None else x, dy, w_shape, stride, padding,
                            want_col=col is None, want_dy2=True)
    col = c2 if col is None else col
    return torch.matmul(dy2, col).view(tuple(w_shape))


def conv_fwd_gemm(x, weight, stride, padding):
    """F.conv2d (no bias, ungrouped) as one fp32 strided-batched library GEMM over the
    im2col matrix, y[n] = W[Co, C*R*S] @ col_n^T (col_n: sample n's P rows), written in
    NCHW directly.  Bit-identical to the one-GEMM y2 = W @ col^T + permute form it replaced
    and 1-4 us faster per ResNet-18 layer3/4 conv (tools/fwd_gemm_layout_probe.py,
    profiles/r3_fwd_gemm_layout.json).  Returns (y, col); col serves the weight gradient."""
    Nb, C_, H, W, Co, R, S, st, pad, OH, OW = _gemm_geo(x.shape, weight.shape, stride, padding)
    col, _ = gemm_operands(x, None, weight.shape, stride, padding, want_col=True, want_dy2=False)
    y = torch.matmul(weight.detach().reshape(Co, C_ * R * S),
                     col.view(Nb, OH * OW, C_ * R * S).transpose(1, 2))
    return y.view(Nb, Co, OH, OW), col


# ------------------------------------------------------------------ K18 depthwise conv
def dwconv_supported(x, weight, stride, padding, dilation, groups):
    """Depthwise shapes K18 handles: fp32 NCHW on the device, groups == C == Co, square
    stride / padding, dilation 1, R*S <= 25, and forward AND input-gradient LDS stages
    (weight rows + padded planes) within the 128 KiB opt-in (ssq_dwconv_supported)."""
    if x.dim() != 4 or weight.dim() != 4 or not x.is_cuda or x.dtype != torch.float32:
        return False
    if groups <= 1 or groups != x.shape[1] or groups != weight.shape[0] or weight.shape[1] != 1:
        return False
    if not isinstance(stride, int) and len(set(stride)) != 1:
        return False
    if not isinstance(padding, int) and (isinstance(padding, str) or len(set(padding)) != 1):
        return False
    if (dilation if isinstance(dilation, int) else max(dilation)) != 1:
        return False
    pad = padding if isinstance(padding, int) else padding[0]
    st = stride if isinstance(stride, int) else stride[0]
    Nb, C, H, W = (int(v) for v in x.shape)
    R, S = int(weight.shape[2]), int(weight.shape[3])
    # both the forward and the input-gradient stage must fit (the planner's own sizes)
    return R * S <= 25 and bool(query("ssq_dwconv_supported", Nb, C, H, W, R, S, int(st), int(pad)))


def _dw_dims(x_shape, w_shape, stride, padding):
    st = stride if isinstance(stride, int) else stride[0]
    pad = padding if isinstance(padding, int) else padding[0]
    Nb, C, H, W = (int(v) for v in x_shape)
    return Nb, C, H, W, int(w_shape[2]), int(w_shape[3]), int(st), int(pad)


def dwconv_fwd(x, weight, stride, padding):
    Nb, C, H, W, R, S, st, pad = _dw_dims(x.shape, weight.shape, stride, padding)
    x, xp = fptr(x.detach(), "x")
    w, wp = fptr(weight.detach(), "weight")
    y = torch.empty((Nb, C, (H + 2 * pad - R) // st + 1, (W + 2 * pad - S) // st + 1),
                    dtype=torch.float32, device=x.device)
    call("ssq_dwconv_fwd", xp, wp, _vp(y), Nb, C, H, W, R, S, st, pad, stream_of(x))
    return y


def dwconv_bwd_data(dy, weight, x_shape, stride, padding):
    Nb, C, H, W, R, S, st, pad = _dw_dims(x_shape, weight.shape, stride, padding)
    dy, dp = fptr(dy.detach(), "dy")
    w, wp = fptr(weight.detach(), "weight")
    dx = torch.empty(tuple(x_shape), dtype=torch.float32, device=dy.device)
    call("ssq_dwconv_bwd_data", dp, wp, _vp(dx), Nb, C, H, W, R, S, st, pad, stream_of(dy))
    return dx


class DwConv2dFn(torch.autograd.Function):
    """Depthwise F.conv2d on K18 (forward, input gradient) and K17's depthwise reduction
    (weight gradient): deterministic, no MIOpen naive kernels."""

    @staticmethod
    def forward(ctx, x, weight, stride, padding):
        ctx.save_for_backward(x, weight)
        ctx.cfg = (stride, padding)
        return dwconv_fwd(x, weight, stride, padding)

    @staticmethod
    def backward(ctx, g):
        x, weight = ctx.saved_tensors
        stride, padding = ctx.cfg
        g = g.contiguous()
        gx = gw = None
        if ctx.needs_input_grad[0]:
            gx = dwconv_bwd_data(g, weight, x.shape, stride, padding)
        if ctx.needs_input_grad[1]:
            gw = conv_wgrad(x, g, weight.shape, stride, padding, int(weight.shape[0]))
        return gx, gw, None, None


def _pair(v):
    return [int(v), int(v)] if isinstance(v, int) else [int(t) for t in v]


class Conv2dFn(torch.autograd.Function):
    """F.conv2d whose weight gradient runs on K17 (deterministic, MFMA) or a library GEMM
    form; the forward and the input gradient stay on MIOpen except where a GEMM form is
    faster (small-plane im2col forwards, 1x1 stride-2 forwards, 1x1 stride-1 input gradients)."""

    @staticmethod
    def forward(ctx, x, weight, stride, padding, dilation, groups, lib_wgrad=False):
        # lib_wgrad: a 1x1 conv taken for its GEMM input gradient only; its weight gradient
        # (if any) stays on MIOpen
        ctx.cfg = (stride, padding, dilation, groups)
        ctx.lib_wgrad = lib_wgrad
        if not lib_wgrad and _use_fwd_gemm(x, weight, stride, padding, groups):
            # small planes: the forward as one library GEMM over the im2col matrix, kept
            # for the weight gradient's GEMM
            y, col = conv_fwd_gemm(x, weight, stride, padding)
            ctx.save_for_backward(x, weight, col)
            return y
        if not lib_wgrad and ctx.needs_input_grad[1] and GROUPED_GEMM_FWD and \
                _use_wgrad_grouped_gemm(x, weight, stride, padding, groups):
            # the im2col matrix the grouped weight gradient reads, built once, forward first
            y, col = conv_fwd_grouped_gemm(x, weight, stride, padding, groups)
            ctx.save_for_backward(x, weight, col)
            return y
        if _use_fwd_1x1(x, weight, stride, padding, dilation, groups):
            y, xs = conv1x1_fwd_gemm(x, weight, stride, keep_xs=True)
            keep = (not lib_wgrad and ctx.needs_input_grad[1]
                    and _use_wgrad_bmm_s2(x, weight, stride, padding, groups))
            ctx.save_for_backward(x, weight, xs if keep else None)
            return y
        ctx.save_for_backward(x, weight, None)
        return torch.nn.functional.conv2d(x, weight, None, stride, padding, dilation, groups)

    @staticmethod
    def backward(ctx, g):
        x, weight, col = ctx.saved_tensors
        stride, padding, dilation, groups = ctx.cfg
        g = g.contiguous()
        gx = gw = None
        if ctx.needs_input_grad[0] and _use_dgrad_1x1(x, weight, stride, padding, groups):
            gx = conv1x1_dgrad_gemm(g, weight)
        elif ctx.needs_input_grad[0]:
            # the saved input itself, not torch.nn.grad.conv2d_input's expanded dummy: the
            # MIOpen backend makes an expanded input contiguous first (one activation-sized
            # copy per call, 8.4 us on a ResNet-18 layer1 batch)
            gx = torch.ops.aten.convolution_backward(
                g, x, weight, None, _pair(stride), _pair(padding), _pair(dilation), False,
                [0, 0], groups, (True, False, False))[0]
        if ctx.needs_input_grad[1] and ctx.lib_wgrad:
            gw = torch.ops.aten.convolution_backward(
                g, x, weight, None, _pair(stride), _pair(padding), _pair(dilation), False,
                [0, 0], groups, (False, True, False))[1]
        elif ctx.needs_input_grad[1]:
            if _use_wgrad_gemm(x, weight, stride, padding, groups):
                gw = conv_wgrad_gemm(x, g, weight.shape, stride, padding, col=col)
            elif _use_wgrad_bmm(x, weight, stride, padding, groups):
                gw = conv_wgrad_1x1_bmm(x, g, weight.shape)
            elif col is not None and _use_wgrad_bmm_s2(x, weight, stride, padding, groups):
                gw = conv_wgrad_1x1_bmm(col, g, weight.shape)   # col: the forward's xs
            elif _use_wgrad_grouped_gemm(x, weight, stride, padding, groups):
                gw = conv_wgrad_grouped_gemm(x, g, weight.shape, stride, padding, groups,
                                             col=col)
            else:
                gw = conv_wgrad(x, g, weight.shape, stride, padding, groups)
        return gx, gw, None, None, None, None, None


# When the conv weight gradient runs on K17 (tools/wgrad_bench.py, batch 32, MI355X,
# profiles/r2_wgrad_band.log):
#   'auto'   every shape the band kernel stages with 16-B pieces (3x3 pad 1: ResNet layer1,
#            layer2, layer3.0's stride-2 conv), in either mode -- it beats MIOpen's fastest
#            non-deterministic solver there (layer1 3x3: 97 vs 110 us, layer2.0 s2: 66 vs
#            81, layer3.0 s2: 66 vs 85); every grouped conv: depthwise ones on K17's
#            LDS-staged reduction (MobileNetV2 144x56x56 3x3: 60 vs 866 us on MIOpen, either
#            mode), other grouped ones on its MFMA GEMM (RegNetX g=2: 326 vs 960 us); under
#            the reference's torch.backends.cudnn.deterministic also every stride-2 conv and
#            every output plane >= 100 pixels, where MIOpen's deterministic solvers are
#            slower (layer3 3x3 14x14: band 132 vs 172 us, layer4.0 s2: 106 vs 372; the
#            7x7 planes of layer4 stay on MIOpen: 98 vs 166).
#   'always' / 'never' (MIOpen's choice) for A/B runs.
WGRAD_POLICY = "auto"


# Conv weight gradients as ONE library GEMM over an im2col matrix (conv_wgrad_gemm) where
# the output plane is small: 3x3 (or larger) ungrouped convs with OH*OW <= 196,
# Co >= 128 and C*R*S >= 1152 -- ResNet-18 layer3 / layer4 (tools/gemm_probe.py,
# profiles/r2_wgrad_gemm.log: the GEMM runs at 94-115 TF there, the band kernel at 57 TF
# on 14x14 planes).  'never' keeps K17 / MIOpen (A/B).
WGRAD_GEMM = "auto"
# ... and the forward of those convs too (MIOpen's deterministic forward takes 99 / 173 us
# on layer3.0 / layer4.0's stride-2 convs where the GEMM takes 42 / 38,
# profiles/r2_wgrad_gemm.log); the im2col matrix is then shared with the weight gradient
WGRAD_GEMM_FWD = True


def _out_plane(x, weight, stride, padding):
    st = stride if isinstance(stride, int) else stride[0]
    pad = padding if isinstance(padding, int) else padding[0]
    oh = (x.shape[2] + 2 * pad - weight.shape[2]) // st + 1
    ow = (x.shape[3] + 2 * pad - weight.shape[3]) // st + 1
    return oh, ow


def _use_wgrad_gemm(x, weight, stride, padding, groups=1):
    # WGRAD_POLICY 'never' is the all-MIOpen A/B mode: no GEMM convs either
    if WGRAD_GEMM != "auto" or WGRAD_POLICY == "never" or groups != 1:
        return False
    if isinstance(stride, (tuple, list)) and len(set(stride)) != 1:
        return False
    if isinstance(padding, str) or (isinstance(padding, (tuple, list)) and len(set(padding)) != 1):
        return False
    oh, ow = _out_plane(x, weight, stride, padding)
    Co, C_, R, S = (int(v) for v in weight.shape)
    NP = x.shape[0] * oh * ow
    if NP * C_ * R * S >= (1 << 31) or Co * NP >= (1 << 31) or oh * ow > 196:
        return False
    if R * S == 1:
        # 1x1 (the ResNet downsamples): layer3.0 / layer4.0 33 / 23 us vs K17's 1x1 kernel
        # 44 / 44; layer2.0's (28x28 plane) stays on K17 (84 vs 42; tools/ds_gemm_probe.py).
        # Under cudnn.deterministic also every 1x1 on a 7x7 plane: MIOpen's deterministic
        # weight gradient takes 74-137 us there (MobileNetV2 960 -> 160: GEMM 25, K17 45;
        # tools/conv1x1_probe.py, profiles/r6_conv1x1_probe.jsonl)
        return Co >= 256 or (oh * ow <= 49 and torch.backends.cudnn.deterministic)
    return Co >= 128 and C_ * R * S >= 1152


# 1x1 stride-1 convs on large planes (OH*OW >= 400: ResNet-50's bottleneck 1x1s and layer1
# downsample, MobileNetV2's expand / project convs, RegNetX's 'a' convs on 28x28 and up): the
# weight gradient as ONE strided-batched library GEMM, sum_n dy[n] @ x[n]^T, then the batch
# summed in order (conv_wgrad_1x1_bmm), instead of K17's 1x1 kernel, whose per-lane 4-B
# LDS-DMA staging holds it at 11-31 TF there.  tools/wgrad1x1_probe.py
# (profiles/r6_wgrad1x1_probe.jsonl), batch 32: ResNet-50 layer1.0 conv1 / conv3 / downsample
# 74.6 / 120.8 / 120.9 -> 20.9 / 35.3 / 35.0 us, RegNetX-3200M s3.b1 'a' 133.7 -> 54.3 us;
# bit-identical run to run, within 1e-6 of float64 (K17: 3e-7).  Planes <= 196 pixels keep
# the im2col GEMM (_use_wgrad_gemm) or K17.  A/B knob: SSQ_WGRAD_1X1_BMM=0.
WGRAD_1X1_BMM = os.environ.get("SSQ_WGRAD_1X1_BMM", "1") != "0"


def _use_wgrad_bmm(x, weight, stride, padding, groups=1):
    if not WGRAD_1X1_BMM or WGRAD_POLICY != "auto" or groups != 1 \
            or tuple(weight.shape[2:]) != (1, 1):
        return False
    if _pair(stride) != [1, 1] or _pair(padding) != [0, 0]:
        return False
    # 14x14 planes too under cudnn.deterministic (MobileNetV2's 14x14 1x1s: 16-27 us vs K17's
    # 39-44; tools/conv1x1_probe.py) where the im2col GEMM does not take them
    p = x.shape[2] * x.shape[3] if x.dim() == 4 else 0
    return p >= 400 or (p >= 100 and torch.backends.cudnn.deterministic)


# The input gradient of 1x1 stride-1 convs as ONE strided-batched library GEMM,
# dx[n] = W^T @ dy[n] (conv1x1_dgrad_gemm), on the shapes where MIOpen's deterministic
# backward-data solver is slower (tools/conv1x1_probe.py over every 1x1 stride-1 conv of
# ResNet-50 / MobileNetV2 / RegNetX-3200M at batch 32, profiles/r6_conv1x1_probe.jsonl):
#   112x112 planes, all (MobileNetV2 16 -> 96: 110 -> 38 us);
#   7x7 planes with Co <= 4 C (ResNet-50 512 -> 2048: 157 -> 37; MobileNetV2 960 -> 160:
#       15.1 -> 12.5; 160 -> 960 is slower as a GEMM, 16.5 -> 41.6);
#   14x14 / 28x28 planes with C >= 128 and Co >= C, and Co >= 2 C on 14x14 (ResNet-50
#       256 -> 1024: 53 -> 35; RegNetX 192 -> 432: 103 -> 51; 432 -> 432 on 14x14 is not);
#   56x56 planes never (the GEMM is 1.3-2.5x slower there).
# A/B knob: SSQ_DGRAD_1X1_GEMM=0.
DGRAD_1X1_GEMM = os.environ.get("SSQ_DGRAD_1X1_GEMM", "1") != "0"


def _use_dgrad_1x1(x, weight, stride, padding, groups=1):
    if not DGRAD_1X1_GEMM or WGRAD_POLICY == "never" or groups != 1 \
            or tuple(weight.shape[2:]) != (1, 1) or not torch.backends.cudnn.deterministic:
        return False
    if _pair(stride) != [1, 1] or _pair(padding) != [0, 0]:
        return False
    if x.dim() != 4 or not x.is_cuda or x.dtype != torch.float32:
        return False
    co, c = int(weight.shape[0]), int(weight.shape[1])
    p = x.shape[2] * x.shape[3]
    if p >= 12544:
        return True
    if p <= 49:
        return co <= 4 * c
    if 196 <= p <= 784:
        return c >= 128 and co >= c and (p >= 784 or co >= 2 * c)
    return False


def conv1x1_dgrad_gemm(dy, weight):
    """d loss / d input of a 1x1 / stride 1 / pad 0 ungrouped conv: W^T @ dy[n] for every
    sample as one strided-batched GEMM (torch.matmul -> hipBLASLt)."""
    n, co, h, w = (int(v) for v in dy.shape)
    c = int(weight.shape[1])
    gx = torch.matmul(weight.detach().reshape(co, c).t(), dy.reshape(n, co, h * w))
    return gx.view(n, c, h, w)


def conv_wgrad_1x1_bmm(x, dy, w_shape):
    """d loss / d weight of a 1x1 / stride 1 / pad 0 ungrouped conv: sum_n dy[n] @ x[n]^T as
    one strided-batched GEMM (torch.matmul -> hipBLASLt) and an in-order batch sum."""
    n, c = int(x.shape[0]), int(x.shape[1])
    co, p = int(w_shape[0]), int(x.shape[2] * x.shape[3])
    gw = torch.matmul(dy.detach().reshape(n, co, p), x.detach().reshape(n, c, p).transpose(1, 2))
    return gw.sum(0).view(tuple(w_shape))


# Grouped (not depthwise) convs on small output planes (OH*OW <= 196: RegNetX-3200M's g = 9 /
# 21 'b' convs of stages 3 and 4): the weight gradient as the im2col operands of every channel
# (ssq_wgrad_gemm_operands) and ONE strided-batched library GEMM over the groups,
# dW[g] = dy2[g rows] @ col[:, g columns] (conv_wgrad_grouped_gemm), instead of K17's implicit
# GEMM, which runs at 6-11 TF there.  tools/wgrad_grouped_probe.py
# (profiles/r6_wgrad_grouped_probe.jsonl), batch 32: s3.b1 268.6 -> 115.5 us, s3.b2 205.4 ->
# 91.0, s4.b1 243.9 -> 70.3, s4.b2 121.7 -> 57.6; on the larger planes of stages 1-2 (g = 2,
# 4) K17 stays faster and keeps them.  Bit-identical run to run, within 1e-6 of float64.
# A/B knob: SSQ_WGRAD_GROUPED_GEMM=0.
WGRAD_GROUPED_GEMM = os.environ.get("SSQ_WGRAD_GROUPED_GEMM", "1") != "0"
# ... and the forward of those convs as one GEMM over the groups on the same im2col matrix,
# built once, in the forward (conv_fwd_grouped_gemm).  A/B knob: SSQ_GROUPED_GEMM_FWD=0.
GROUPED_GEMM_FWD = os.environ.get("SSQ_GROUPED_GEMM_FWD", "1") != "0"


def _use_wgrad_grouped_gemm(x, weight, stride, padding, groups=1):
    if not WGRAD_GROUPED_GEMM or WGRAD_POLICY != "auto" or groups <= 1 or weight.shape[1] <= 1:
        return False
    if isinstance(stride, (tuple, list)) and len(set(stride)) != 1:
        return False
    if isinstance(padding, str) or (isinstance(padding, (tuple, list)) and len(set(padding)) != 1):
        return False
    oh, ow = _out_plane(x, weight, stride, padding)
    Co, Cig, R, S = (int(v) for v in weight.shape)
    NP = x.shape[0] * oh * ow
    if NP * Cig * groups * R * S >= (1 << 31) or Co * NP >= (1 << 31):
        return False
    return oh * ow <= 196


def conv_wgrad_grouped_gemm(x, dy, w_shape, stride, padding, groups, col=None):
    """d loss / d weight of a grouped conv: the im2col matrix of every input channel and the
    permuted gradient (ssq_wgrad_gemm_operands, as for an ungrouped conv of C_in = Cig * G),
    then one strided-batched GEMM over the groups (group g: its Cog rows of dy2 against its
    Cig * R * S columns of col).  col may be the forward's (conv_fwd_grouped_gemm), saved."""
    Co, Cig, R, S = (int(v) for v in w_shape)
    c2, dy2 = gemm_operands(x, dy, (Co, Cig * groups, R, S), stride, padding,
                            want_col=col is None, want_dy2=True)
    col = c2 if col is None else col
    NP = col.shape[0]
    a = dy2.view(groups, Co // groups, NP)
    b = col.view(NP, groups, Cig * R * S).transpose(0, 1)
    return torch.matmul(a, b).reshape(tuple(w_shape))


def conv_fwd_grouped_gemm(x, weight, stride, padding, groups):
    """F.conv2d of a grouped conv (no bias) on _use_wgrad_grouped_gemm's shapes as the im2col
    matrix of every input channel (the one its weight gradient reads: returned, to be saved)
    and ONE strided-batched GEMM over the groups, Y[g] = W[g] @ col[:, g]^T (G x Cog x N*P),
    then permuted to NCHW.  RegNetX-3200M s3.b1's 'b' conv (g = 9, stride 2): MIOpen's
    deterministic forward 102.5 us; here the im2col build moves from the backward to the
    forward (tools/recon_configs_trace.py).  Returns (y, col)."""
    Nb, C_, H, W, Co, R, S, st, pad, OH, OW = _gemm_geo(x.shape, weight.shape, stride, padding)
    C_ = int(weight.shape[1]) * groups
    k = int(weight.shape[1]) * R * S
    col, _ = gemm_operands(x, None, (Co, C_, R, S), stride, padding, want_col=True,
                           want_dy2=False)
    y = torch.matmul(weight.detach().reshape(groups, Co // groups, k),
                     col.view(-1, groups, k).permute(1, 2, 0))
    y = y.view(groups, Co // groups, Nb, OH * OW).permute(2, 0, 1, 3).contiguous()
    return y.view(Nb, Co, OH, OW), col


def _use_fwd_gemm(x, weight, stride, padding, groups=1):
    """The forward as the im2col GEMM on the weight-gradient GEMM's shapes.  Extending it to
    layer2.0's stride-2 conv (MIOpen's deterministic forward 99 us standalone, the GEMM 40
    + the 58 MB im2col pass) measured no gain in the loop (1639 -> 1617 it/s,
    profiles/r2_wgrad_gemm.log), so it is not."""
    return (WGRAD_GEMM_FWD and weight.shape[2] * weight.shape[3] > 1
            and _use_wgrad_gemm(x, weight, stride, padding, groups))


# 1x1 stride-2 convs (the ResNet downsamples) forward as ONE strided-batched library GEMM
# on the subsampled input, y[n] = W @ x[n, :, ::s, ::s]: NCHW in, NCHW out (MIOpen
# transposes NCHW <-> CNHW around its own GEMM).  tools/ds_fwd_probe.py
# (profiles/r3_ds_fwd_probe.json), deterministic solvers: layer2.0 35.9 -> 22.3 us and
# layer4.0 30.9 -> 14.4 at batch 32 (recon), 112 -> 66 and 103 -> 34 at batch 128
# (validation); layer3.0's 14x14 plane is slower at batch 32 (27.5 -> 56.6, hipBLASLt's
# pick for that batched shape), so output planes of 100-400 pixels stay on MIOpen below
# batch 128.  Bit-identical run to run.  Stride-1 1x1 convs stay on MIOpen (unmeasured).
# A/B knob: SSQ_FWD_1X1_GEMM=0.
FWD_1X1_GEMM = os.environ.get("SSQ_FWD_1X1_GEMM", "1") != "0"


def _use_fwd_1x1(x, weight, stride, padding, dilation, groups):
    # WGRAD_POLICY 'never' is the all-MIOpen A/B mode: no GEMM convs there either
    if not FWD_1X1_GEMM or WGRAD_POLICY == "never" or groups != 1 or weight.shape[2] != 1 \
            or weight.shape[3] != 1:
        return False
    if x.dim() != 4 or not x.is_cuda or x.dtype != torch.float32:
        return False
    st, pad, dil = (_pair(v) for v in (stride, padding, dilation))
    if st[0] != st[1] or st[0] < 2 or pad != [0, 0] or dil != [1, 1]:
        return False
    oh, ow = _out_plane(x, weight, st[0], 0)
    return not (100 < oh * ow < 400 and x.shape[0] < 128)


def conv1x1_fwd_gemm(x, weight, stride, keep_xs=False):
    """F.conv2d of a 1x1 / pad 0 / stride s conv as one strided-batched GEMM on the
    subsampled input (see FWD_1X1_GEMM); keep_xs: also return that input, contiguous (the
    weight gradient's operand, conv_wgrad_1x1_bmm)."""
    st = stride if isinstance(stride, int) else stride[0]
    xs = x[:, :, ::st, ::st].contiguous()
    n, c, oh, ow = xs.shape
    co = int(weight.shape[0])
    y = torch.matmul(weight.detach().reshape(co, c), xs.view(n, c, oh * ow))
    y = y.view(n, co, oh, ow)
    return (y, xs) if keep_xs else y


# 1x1 stride-2 weight gradients on output planes >= 400 pixels (the forward GEMM above made
# the subsampled input contiguous) with channel counts in whole 64s: one strided-batched GEMM
# + batch sum over that input (conv_wgrad_1x1_bmm) instead of K17's 1x1 kernel.
# tools/ds_wgrad_probe.py (profiles/r6_ds_wgrad_probe.jsonl), batch 32: ResNet-18 layer2.0
# 41.1 -> 31.6 us, ResNet-50 layer2.0 138.9 -> 65.3; RegNetX s2.b1 (96 -> 192) is slower as
# the GEMM (79.3 vs 43.6) and keeps K17; on 14x14 and 7x7 planes the im2col GEMM stays.
# A/B knob: SSQ_WGRAD_S2_BMM=0.
WGRAD_S2_BMM = os.environ.get("SSQ_WGRAD_S2_BMM", "1") != "0"


def _use_wgrad_bmm_s2(x, weight, stride, padding, groups=1):
    if not WGRAD_S2_BMM or WGRAD_POLICY != "auto" or groups != 1 \
            or tuple(weight.shape[2:]) != (1, 1) or _pair(padding) != [0, 0]:
        return False
    st = _pair(stride)
    if st[0] != st[1] or st[0] < 2:
        return False
    oh, ow = _out_plane(x, weight, st[0], 0)
    co, c = int(weight.shape[0]), int(weight.shape[1])
    return oh * ow >= 400 and c % 64 == 0 and co % 64 == 0


def _use_k17(x, weight, stride, padding, groups=1):
    if WGRAD_POLICY == "always":
        return True
    if WGRAD_POLICY != "auto":
        return False
    if groups > 1:
        return True
    if _use_wgrad_gemm(x, weight, stride, padding, groups):
        return True
    if wgrad_kind(x.shape, weight.shape, stride, padding, groups) == 3:
        return True
    if torch.backends.cudnn.deterministic:
        st = stride if isinstance(stride, int) else stride[0]
        pad = padding if isinstance(padding, int) else padding[0]
        oh = (x.shape[2] + 2 * pad - weight.shape[2]) // st + 1
        ow = (x.shape[3] + 2 * pad - weight.shape[3]) // st + 1
        return st > 1 or oh * ow >= 100
    return False


# Depthwise convs on K18 + K17 ('auto'; MIOpen runs them on naive direct kernels) or on
# MIOpen ('never').
DWCONV_POLICY = "auto"


def conv2d(x, weight, stride=1, padding=0, dilation=1, groups=1):
    """F.conv2d without bias: depthwise convs on K18/K17 (DWCONV_POLICY), otherwise MIOpen
    with the K17 weight gradient when the weight needs one (WGRAD_POLICY); 1x1 stride-2
    forwards as one batched GEMM (FWD_1X1_GEMM); a LazyEpi input (a BasicBlock's conv1
    epilogue) folded into the im2col GEMM of conv_fwd_gemm's shapes, else materialised."""
    if getattr(x, "_ssq_epi", None) is not None:
        if (weight.requires_grad and torch.is_grad_enabled() and groups == 1 and
                (dilation if isinstance(dilation, int) else max(dilation)) == 1 and
                _use_fwd_gemm(x, weight, stride, padding, groups)):
            return epi_conv_gemm(x, weight, stride, padding)
        x = materialize_epi(x)
    if DWCONV_POLICY == "auto" and dwconv_supported(x, weight, stride, padding, dilation, groups) \
            and x.is_contiguous():
        if torch.is_grad_enabled() and (x.requires_grad or weight.requires_grad):
            return DwConv2dFn.apply(x, weight, stride, padding)
        return dwconv_fwd(x, weight, stride, padding)
    if weight.requires_grad and torch.is_grad_enabled() and \
            (dilation if isinstance(dilation, int) else max(dilation)) == 1 and \
            (_use_wgrad_gemm(x, weight, stride, padding, groups) or
             _use_wgrad_grouped_gemm(x, weight, stride, padding, groups) or
             (conv_wgrad_supported(x, weight, stride, padding, dilation, groups) and
              _use_k17(x, weight, stride, padding, groups))):
        return Conv2dFn.apply(x, weight, stride, padding, dilation, groups)
    if torch.is_grad_enabled() and x.requires_grad and \
            _use_dgrad_1x1(x, weight, stride, padding, groups):
        # a 1x1 conv K17 does not take (an activation-phase conv, or a small plane): its
        # input gradient as a GEMM, its weight gradient (if any) on MIOpen as before
        return Conv2dFn.apply(x, weight, stride, padding, dilation, groups, True)
    if _use_fwd_1x1(x, weight, stride, padding, dilation, groups) and \
            not (torch.is_grad_enabled() and (x.requires_grad or weight.requires_grad)):
        return conv1x1_fwd_gemm(x, weight, stride)
    return torch.nn.functional.conv2d(x, weight, None, stride, padding, dilation, groups)
