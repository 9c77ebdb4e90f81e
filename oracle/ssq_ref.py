"""CPU oracle: a numpy restatement of the reference's shifted-scale quantization path.

TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg may import this module, and only as the checker / CPU baseline.
The product path (shiftedscalequantization_amd) never imports it and fails loudly
when its HIP library is missing.

Every function restates one piece of the reference (jai1215snu/ShiftedScaleQuantization,
cited as file:line under /root/reference) with the reference's own fp32 operation
order, so that integer codes are bit-exact.  Parity is PINNED: tests/test_oracle.py
checks each function against the golden vectors in tests/golden/*.npz, which were
produced by running the reference itself (tests/golden/make_golden.py).

Scalar semantics of the reference (PyTorch CPU, fp32 tensors):
  * tensor (op) python_float  -> the float is first rounded to fp32, then one fp32 op;
  * python_float / tensor     -> Tensor.__rtruediv__ = reciprocal(tensor) * float;
  * torch.round               -> round-half-to-even (np.rint);
  * clamp backward mask       -> inclusive on both bounds.
Reductions (sums / means) are accumulated in float64 here; the reference's own
summation order is not reproducible, so reduced values are compared with a
relative tolerance in the tests, never the integer codes.
"""
import numpy as np

F32 = np.float32
GAMMA = F32(-0.1)                         # channelQuant.py:35, adaptive_rounding.py:31
ZETA = F32(1.1)
ZMG = F32(1.1 - (-0.1))                   # (zeta - gamma) python float 1.2000000000000002 -> fp32


def _f(x):
    return np.asarray(x, dtype=F32)


def qrange(n_bits, sym):
    n = 2 ** n_bits
    return (-(n // 2), n // 2 - 1) if sym else (0, n - 1)


# ----------------------------------------------------------------- K1 / K2  (quant_layer.py:77-98)
def round_ste_fwd(t):
    """round_ste's forward value (quant_layer.py:18-22): (round(t) - t) + t in fp32 --
    round(t) for every finite t, NaN at t = +-inf."""
    t = _f(t)
    with np.errstate(invalid="ignore"):
        return ((np.rint(t) - t) + t).astype(F32)


def fake_quant(x, delta, zp, n_bits, sym=False, ste=True):
    """UniformAffineQuantizer.forward (quant_layer.py:92-98). delta/zp broadcast against x.
    ste=False: plain torch.round (ChannelQuant / ChannelQuantAct 'none').  np.clip keeps
    NaN, as torch.clamp.  Returns (dequantized fp32, integer codes as int32)."""
    x, delta, zp = _f(x), _f(delta), _f(zp)
    lo, hi = qrange(n_bits, sym)
    with np.errstate(invalid="ignore", over="ignore", divide="ignore"):
        t = x / delta
        x_int = (round_ste_fwd(t) if ste else np.rint(t)) + zp
        xq = np.clip(x_int, F32(lo), F32(hi))
        codes = np.where(np.isnan(xq), F32(0), xq).astype(np.int32)
        return ((xq - zp) * delta).astype(F32), codes


def fake_quant_bwd(x, delta, zp, n_bits, sym, gy):
    """Autograd of quant_layer.py:92-98 (STE).  Returns gx, gdelta, gzp (gdelta/gzp with
    delta's broadcast shape, summed in float64)."""
    x, delta, zp, gy = _f(x), _f(delta), _f(zp), _f(gy)
    lo, hi = qrange(n_bits, sym)
    t = x / delta
    x_int = round_ste_fwd(t) + zp
    m = (x_int >= lo) & (x_int <= hi)
    xq = np.clip(x_int, F32(lo), F32(hi))
    g_q = gy * delta                                  # mul backward (wrt x_quant - zp)
    g_int = np.where(m, g_q, F32(0))                  # clamp backward
    gx = (g_int / delta).astype(F32)                  # div backward wrt x
    gd_mul = (gy.astype(np.float64) * (xq - zp))      # mul backward wrt delta
    gd_div = -(g_int.astype(np.float64)) * ((t / delta).astype(np.float64))  # div backward wrt delta
    red = tuple(i for i in range(x.ndim) if delta.ndim == 0 or delta.shape[i] == 1) \
        if delta.ndim else tuple(range(x.ndim))
    gdelta = (gd_mul.sum(axis=red, keepdims=True) + gd_div.sum(axis=red, keepdims=True))
    gzp = (g_int.astype(np.float64).sum(axis=red, keepdims=True)
           - g_q.astype(np.float64).sum(axis=red, keepdims=True))
    return gx, gdelta.reshape(delta.shape), gzp.reshape(zp.shape)


# ----------------------------------------------------------------- K3 / K4  (quant_layer.py:100-175)
def _py_round(v):
    """Python's round(): half-to-even on a double; round(nan) raises ValueError (the
    reference's 'max' init on a NaN row or x_min = -inf, quant_layer.py:140)."""
    if np.isnan(v):
        raise ValueError("cannot convert float NaN to integer")
    return float(np.rint(v))


def init_scale_max(row, n_bits, sym=False, scale=False):
    """'max' branch, quant_layer.py:124-142 (host fp64 math on fp32 min/max)."""
    row = _f(row)
    x_min = min(float(row.min()), 0.0)
    x_max = max(float(row.max()), 0.0)
    if scale:
        x_min = x_min * (n_bits + 2) / 8
        x_max = x_max * (n_bits + 2) / 8
    if sym:
        x_absmax = max(abs(x_min), x_max)
        x_min, x_max = (-x_absmax if x_min < 0 else 0), x_absmax
    delta = float(x_max - x_min) / (2 ** n_bits - 1)
    if delta < 1e-8:
        delta = 1e-8
    zero_point = _py_round(-x_min / delta)
    return F32(delta), F32(zero_point), F32(-x_min)


def _quantize_cand(x, mx, mn, n_bits):
    """UniformAffineQuantizer.quantize, quant_layer.py:168-175 (fp32)."""
    delta = (mx - mn) / F32(2 ** n_bits - 1)
    zp = np.rint(-mn / delta)
    x_int = np.rint(x / delta)
    xq = np.clip(x_int + zp, F32(0), F32(2 ** n_bits - 1))
    return (xq - zp) * delta


def init_scale_mse(x, n_bits, sym=False, return_scores=False):
    """'mse' branch, quant_layer.py:144-162: 80 shrink candidates, Lp(2.4) score, first strict min."""
    with np.errstate(all="ignore"):   # constant / infinite rows: x/0, inf/inf -> NaN scores
        return _init_scale_mse(_f(x), n_bits, sym, return_scores)


def _init_scale_mse(x, n_bits, sym, return_scores):
    x_max, x_min = F32(x.max()), F32(x.min())
    if sym:
        x_absmax = max(abs(x_min), x_max)
        x_min, x_max = (F32(-x_absmax) if x_min < 0 else F32(0)), F32(x_absmax)
    best = 1e10
    delta = zp = raw = None
    scores = []
    for i in range(80):
        s = F32(1.0 - (i * 0.01))
        new_max, new_min = F32(x_max * s), F32(x_min * s)
        xq = _quantize_cand(x, new_max, new_min, n_bits)
        score = float(np.mean(np.abs(x - xq).astype(np.float64) ** 2.4))
        scores.append(score)
        if score < best:
            best = score
            delta = F32((new_max - new_min) / F32(2 ** n_bits - 1))
            zp = F32(np.rint(-new_min / delta)) if not sym else F32(0)
            raw = F32(-new_min) if not sym else F32(0)
    if return_scores:
        return delta, zp, raw, np.array(scores)
    return delta, zp, raw


def init_scale(x, n_bits, sym=False, channel_wise=False, method="max"):
    """init_quantization_scale, quant_layer.py:100-122 (per row when channel_wise)."""
    x = _f(x)
    fn = init_scale_max if "max" in method else init_scale_mse
    kw = {"scale": "scale" in method} if "max" in method else {}
    if channel_wise:
        rows = x.reshape(x.shape[0], -1)
        res = [fn(r, n_bits, sym, **kw) for r in rows]
        if any(v[0] is None for v in res):
            # 'mse' found no candidate for a row: the reference assigns its None delta into
            # the channel's slot, a TypeError (quant_layer.py:114)
            raise TypeError("a row has no 'mse' quantization scale (delta None)")
        shape = (-1,) + (1,) * (x.ndim - 1)
        d, z, r = (np.array([v[i] for v in res], F32).reshape(shape) for i in range(3))
        return d, z, r
    d, z, r = fn(x, n_bits, sym, **kw)
    if d is None:
        return None, None, None   # per-tensor 'mse' without a candidate: the reference's None
    return F32(d), F32(z), F32(r)


# ----------------------------------------------------------------- soft targets (channelQuant.py:120-127)
def softmax(a, axis=-1):
    a = _f(a)
    e = np.exp((a - a.max(axis=axis, keepdims=True)).astype(np.float64))
    return (e / e.sum(axis=axis, keepdims=True)).astype(F32)


def sig_soft_targets(alpha):
    """get_sig_soft_targets, channelQuant.py:120-121."""
    return np.clip(softmax(alpha) * ZMG + GAMMA, F32(0), F32(1))


def sigmoid(v):
    v = _f(v).astype(np.float64)
    return (1.0 / (1.0 + np.exp(-v))).astype(F32)


def soft_round(beta):
    """get_soft_round / get_soft_targets, channelQuant.py:123-127, adaptive_rounding.py:63-64."""
    return np.clip(sigmoid(beta) * ZMG + GAMMA, F32(0), F32(1))


def _rect_sigmoid_inverse(rest):
    """-log((zeta-gamma)/(rest-gamma) - 1): python_float / tensor is reciprocal(tensor)*float
    (channelQuant.py:292,306, adaptive_rounding.py:70)."""
    rest = _f(rest)
    den = rest - GAMMA
    r = (F32(1) / den) * ZMG
    return (-np.log((r - F32(1)).astype(np.float64))).astype(F32)


# ----------------------------------------------------------------- K9  shift init (channelQuant.py:158-307)
def shift_floors(w, delta, shifts):
    """x_q[i] = floor(x / (delta * s_i)), channelQuant.py:284-286."""
    w, delta = _f(w), _f(delta)
    return [np.floor(w / (delta * F32(s))).astype(F32) for s in shifts]


def inverse_softmax(prob):
    """channelQuant.py:193-199."""
    x = (_f(prob) - GAMMA) / ZMG
    logits = np.log(x.astype(np.float64)).astype(F32)
    return (logits - logits.mean(axis=-1, keepdims=True, dtype=np.float64).astype(F32)).astype(F32)


def init_alpha(w, xq, is_fc):
    """init_alpha, channelQuant.py:158-191 (clip forced to 0.33)."""
    w = _f(w)
    S = len(xq)
    if is_fc:
        mse = np.stack([((w - q) ** 2).astype(np.float64) for q in xq])
    else:
        mse = np.stack([((w - q) ** 2).astype(np.float64).sum(axis=(0, 2, 3)) for q in xq])
    min_index = np.argmin(mse, axis=0)
    clip, remain = (1.0, 0.0) if S == 1 else (0.33, (1.0 - 0.33) / (S - 1))
    prob = np.full(min_index.shape + (S,), F32(remain), dtype=F32)
    for i in range(S):
        prob[..., i][min_index == i] = F32(clip)
    return inverse_softmax(prob), min_index


def get_delta(delta, alpha, shifts, is_fc):
    """get_delta, channelQuant.py:221-237: delta * s[argmax p] (first index on ties)."""
    delta = _f(delta)
    p = sig_soft_targets(alpha)
    if p.ndim == 2:
        p = p[None]
    idx = np.argmax(p, axis=-1)
    if not is_fc:
        idx = idx[..., None, None]
    out = delta * F32(shifts[0])
    for i in range(1, len(shifts)):
        out = np.where(idx == i, delta * F32(shifts[i]), out)
    return out.astype(F32)


def init_beta_from_delta(w, delta):
    """beta = -log((zeta-gamma)/(rest-gamma)-1), channelQuant.py:300-307 / :289-292."""
    w, delta = _f(w), _f(delta)
    t = w / delta
    rest = t - np.floor(t)
    return _rect_sigmoid_inverse(rest)


def init_v_beta(w, delta, shifts):
    """channelQuant.py:279-294. Returns (x_q floors list, alpha, beta)."""
    w = _f(w)
    is_fc = w.ndim != 4
    xq = shift_floors(w, delta, shifts)
    alpha, _ = init_alpha(w, xq, is_fc)
    dsel = get_delta(delta, alpha, shifts, is_fc)
    beta = init_beta_from_delta(w, dsel)
    return xq, alpha, beta


def none_fwd(w, delta, zp, n_bits, sym, scale=1.0):
    """ChannelQuant.forward 'none', channelQuant.py:79-94."""
    w, delta, zp = _f(w), _f(delta), _f(zp)
    lo, hi = qrange(n_bits, sym)
    d = delta * F32(scale)
    x_int = np.rint(w / d)
    xq = np.clip(x_int + zp, F32(lo), F32(hi)) - zp
    return (xq * d).astype(F32)


def init_v(w, delta, zp, n_bits, sym, shifts):
    """channelQuant.py:201-213: dequantized candidates + alpha."""
    w = _f(w)
    xq = [none_fwd(w, delta, zp, n_bits, sym, s) for s in shifts]
    alpha, _ = init_alpha(w, xq, w.ndim != 4)
    return xq, alpha


# ----------------------------------------------------------------- K5-K8 forward/backward
def _p_broadcast(p, is_fc):
    if p.ndim == 2:
        p = p[None]
    if not is_fc:
        p = p[..., None, None]           # (1,Ci,S,1,1)
    return p


def shifted_x_quant(xq, alpha, is_fc, hard_targets):
    """channelQuant.py:96-118."""
    p = sig_soft_targets(alpha)
    S = len(xq)
    if hard_targets:
        pp = p[None] if p.ndim == 2 else p
        idx = np.argmax(pp, axis=-1)
        if not is_fc:
            idx = idx[..., None, None]
        out = xq[0]
        for i in range(1, S):
            out = np.where(idx == i, xq[i], out)
        return out.astype(F32)
    P = _p_broadcast(p, is_fc)
    out = xq[0] * (P[:, :, 0] if is_fc else P[:, :, 0, :, :])
    for i in range(1, S):
        out = out + xq[i] * (P[:, :, i] if is_fc else P[:, :, i, :, :])
    return out.astype(F32)


def adashift_fwd(xq, alpha, beta, delta, zp, n_bits, sym, is_fc, hard_targets, hard_round):
    """ChannelQuant.forward 'adaShift', channelQuant.py:51-64."""
    lo, hi = qrange(n_bits, sym)
    delta, zp = _f(delta), _f(zp)
    x_floor = shifted_x_quant(xq, alpha, is_fc, hard_targets)
    if hard_round:
        x_int = x_floor + (_f(beta) >= 0).astype(F32)
    else:
        x_int = x_floor + soft_round(beta)
    xqt = np.clip(x_int + zp, F32(lo), F32(hi))
    return ((xqt - zp) * (delta * F32(1.0))).astype(F32)


def _softmax_clamp_bwd(alpha, g_p):
    """Backward through clamp(softmax(a)*c+gamma, 0, 1), channelQuant.py:120-121."""
    s = softmax(alpha)
    u = s * ZMG + GAMMA
    m = (u >= 0) & (u <= 1)
    g_s = (np.where(m, g_p, 0.0) * float(ZMG)).astype(np.float64)
    s64 = s.astype(np.float64)
    return s64 * (g_s - (g_s * s64).sum(axis=-1, keepdims=True))


def adashift_bwd(xq, alpha, beta, delta, zp, n_bits, sym, is_fc, hard_round, gy):
    """Autograd of adaShift soft-target forward wrt alpha (and beta when soft round).
    Returns (galpha fp64, gbeta fp32 or None)."""
    lo, hi = qrange(n_bits, sym)
    delta, zp, gy = _f(delta), _f(zp), _f(gy)
    x_floor = shifted_x_quant(xq, alpha, is_fc, False)
    h = None if hard_round else soft_round(beta)
    x_int = x_floor + ((_f(beta) >= 0).astype(F32) if hard_round else h)
    v = x_int + zp
    m = (v >= lo) & (v <= hi)
    g_int = np.where(m, gy * (delta * F32(1.0)), F32(0)).astype(np.float64)
    S = len(xq)
    if is_fc:
        g_p = np.stack([g_int * xq[i] for i in range(S)], axis=-1)           # (Co,Ci,S)
    else:
        g_p = np.stack([(g_int * xq[i]).sum(axis=(0, 2, 3)) for i in range(S)], axis=-1)  # (Ci,S)
    g_p = g_p.reshape(_f(alpha).shape)
    galpha = _softmax_clamp_bwd(alpha, g_p)
    gbeta = None
    if not hard_round:
        sg = sigmoid(beta)
        u = sg * ZMG + GAMMA
        mm = (u >= 0) & (u <= 1)
        gbeta = (np.where(mm, g_int, 0.0) * float(ZMG) * (1.0 - sg) * sg).astype(F32)
    return galpha, gbeta


def lhs_bwd(xq, alpha, is_fc, gy):
    """Autograd of 'learned_hard_sigmoid' soft forward (channelQuant.py:81-82) wrt alpha."""
    gy = _f(gy).astype(np.float64)
    S = len(xq)
    if is_fc:
        g_p = np.stack([gy * xq[i] for i in range(S)], axis=-1)
    else:
        g_p = np.stack([(gy * xq[i]).sum(axis=(0, 2, 3)) for i in range(S)], axis=-1)
    return _softmax_clamp_bwd(alpha, g_p.reshape(_f(alpha).shape))


def adaround_fwd(w, beta, delta, zp, n_bits, sym, hard_round, scale=1.0):
    """ChannelQuant 'adaround' (channelQuant.py:65-78) == AdaRoundQuantizer
    'learned_hard_sigmoid' (adaptive_rounding.py:55-67) for scale 1, asym."""
    lo, hi = qrange(n_bits, sym)
    w, delta, zp = _f(w), _f(delta), _f(zp)
    d = delta * F32(scale)
    x_floor = np.floor(w / d)
    x_int = x_floor + ((_f(beta) >= 0).astype(F32) if hard_round else soft_round(beta))
    xq = np.clip(x_int + zp, F32(lo), F32(hi))
    return ((xq - zp) * d).astype(F32)


def adaround_bwd(w, beta, delta, zp, n_bits, sym, gy, scale=1.0):
    """d/dbeta of the soft adaround forward."""
    lo, hi = qrange(n_bits, sym)
    w, delta, zp, gy = _f(w), _f(delta), _f(zp), _f(gy)
    d = delta * F32(scale)
    h = soft_round(beta)
    v = np.floor(w / d) + h + zp
    m = (v >= lo) & (v <= hi)
    g_h = np.where(m, gy * d, F32(0)).astype(np.float64)
    sg = sigmoid(beta).astype(np.float64)
    u = sigmoid(beta) * ZMG + GAMMA
    mm = (u >= 0) & (u <= 1)
    return (np.where(mm, g_h, 0.0) * float(ZMG) * (1.0 - sg) * sg).astype(F32)


# ----------------------------------------------------------------- K10  (channelQuantMSE.py:203-276)
def inpscale_search(w, delta, raw_zp, n_bits, level, threshold):
    """ChannelQuantMSE.init_scale 'max' mode: per (Ci,kh,kw) the LAST candidate c
    (level/level ... 1/level) whose normalized code range over Co fits the limits."""
    w, delta, raw_zp = _f(w), _f(delta), _f(raw_zp)
    x_range = 2 ** n_bits - 1
    min_lim = 0.0 - 0.5 / x_range * threshold
    max_lim = 1.0 + 0.5 / x_range * threshold
    zero = np.rint(raw_zp / delta)
    inp = np.ones((1,) + w.shape[1:], F32)
    for k in range(level, 0, -1):
        c = F32(k / level)
        xq = ((w / c) / delta + zero) / F32(x_range)
        mn, mx = xq.min(axis=0, keepdims=True), xq.max(axis=0, keepdims=True)
        ok = (mn > F32(min_lim)) & (mx < F32(max_lim))
        inp = np.where(ok, c, inp)
    return inp.astype(F32)


def inpscale_fwd(w, inp, delta, raw_zp, n_bits):
    """ChannelQuantMSE.forward, channelQuantMSE.py:267-276."""
    w, inp, delta, raw_zp = _f(w), _f(inp), _f(delta), _f(raw_zp)
    zp = np.rint(raw_zp / delta)
    x_int = np.rint((w / inp) / delta) + zp
    xq = np.clip(x_int, F32(0), F32(2 ** n_bits - 1)) - zp
    return ((xq * delta) * inp).astype(F32)


# ----------------------------------------------------------------- K11 / K12  losses
def lp_loss(pred, tgt, p=2.0, reduction="none"):
    """quant_layer.py:25-32 (+ its autograd wrt pred).  Returns (loss float64, grad fp32)."""
    pred, tgt = _f(pred), _f(tgt)
    d = (pred - tgt).astype(F32)
    a = np.abs(d).astype(np.float64)
    if reduction == "none":
        M = d.size // d.shape[1]
        loss = (a ** p).sum() / M
    else:
        M = d.size
        loss = (a ** p).mean()
    g = F32(1.0) / F32(M)
    ga = (np.float64(g) * (p * a ** (p - 1))) if p != 1 else np.full_like(a, np.float64(g))
    grad = (ga * np.sign(d)).astype(F32)
    return float(loss), grad


def round_reg(vals, b, lmda):
    """lmda * sum(1 - |2v-1|^b) and its gradient wrt v (layer_recon_fused_shiftedScale.py:277-282,
    block_recon.py:171-174)."""
    v = _f(vals).astype(np.float64)
    r = np.abs(v - 0.5) * 2
    loss = lmda * (1 - r ** b).sum()
    if b == 0:
        return float(loss), np.zeros_like(v)
    grad = -lmda * b * r ** (b - 1) * 2 * np.sign(v - 0.5)
    return float(loss), grad


def reg_shift(alpha, b, lmda):
    """Shift regulariser on p(alpha) and its gradient wrt alpha."""
    loss, g_p = round_reg(sig_soft_targets(alpha), b, lmda)
    return loss, _softmax_clamp_bwd(alpha, g_p)


def reg_round(beta, b, lmda):
    """Rounding regulariser on h(beta) and its gradient wrt beta."""
    h = soft_round(beta)
    loss, g_h = round_reg(h, b, lmda)
    sg = sigmoid(beta).astype(np.float64)
    u = sigmoid(beta) * ZMG + GAMMA
    mm = (u >= 0) & (u <= 1)
    return loss, np.where(mm, g_h, 0.0) * float(ZMG) * (1.0 - sg) * sg


def reg_entropy(alpha, lmda):
    """lmda * -sum(p log(p+1e-10)), layer_recon_shiftedScale.py:393,467."""
    p = sig_soft_targets(alpha).astype(np.float64)
    loss = lmda * -(p * np.log(p + 1e-10)).sum()
    g_p = -lmda * (np.log(p + 1e-10) + p / (p + 1e-10))
    return float(loss), _softmax_clamp_bwd(alpha, g_p)


def linear_temp_decay(t, t_max, rel_start_decay=0.2, start_b=20, end_b=2, guard_zero=False):
    """LinearTempDecay (block_recon.py:185-202) / LinearTempDecayShift / FusedLinearTempDecayShift
    (layer_recon_fused_shiftedScale.py:382-399, which guards t_max == 0)."""
    start_decay = rel_start_decay * t_max
    if t < start_decay:
        return start_b
    if guard_zero and t_max == 0:
        rel_t = 1
    else:
        rel_t = (t - start_decay) / (t_max - start_decay)
    return end_b + (start_b - end_b) * max(0.0, (1 - rel_t))


# ----------------------------------------------------------------- K14 gather
def gather_rows(src, idx):
    """cached_inp[permIdx] (layer_recon_fused_shiftedScale.py:95-97)."""
    return np.ascontiguousarray(_f(src)[np.asarray(idx)])
