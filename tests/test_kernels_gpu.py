"""HIP kernel parity through the C ABI: golden fixtures (reference outputs) and the CPU
oracle on seeded inputs.  Integer codes and all-integer dequant paths are bit-exact;
values through transcendentals / reductions use the tolerances written below."""
import numpy as np
import pytest
import torch

from oracle import ssq_ref as R

pytestmark = pytest.mark.gpu

SHIFTS = [31 / 32, 33 / 32, 1.0]


@pytest.fixture(scope="module")
def K():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from shiftedscalequantization_amd import kernels
    return kernels


def dev(a):
    return torch.as_tensor(np.asarray(a, np.float32)).cuda()


def host(t):
    return t.detach().float().cpu().numpy()


def close(a, b, rtol=1e-5, atol=1e-6):
    np.testing.assert_allclose(np.asarray(a, np.float64), np.asarray(b, np.float64), rtol=rtol, atol=atol)


def tags(g, suffix):
    return sorted(k[: -len(suffix)] for k in g if k.endswith(suffix))


# ------------------------------------------------------------------ K1-K4 on goldens
def test_uaq_golden(K, golden):
    g = golden("uaq")
    for t in tags(g, "_gdelta"):
        bits = int(t.split("_")[0][1:])
        sym = "_sym_" in t
        cw = "_cw_" in t
        method = t.rsplit("_", 1)[1]
        x = dev(g[t + "_x"])
        d, z, r = K.scale_init(x, bits, sym, cw, method)
        np.testing.assert_array_equal(host(d).reshape(-1), g[t + "_delta"], err_msg=t)
        np.testing.assert_array_equal(host(z).reshape(-1), g[t + "_zp"], err_msg=t)
        y, codes = K.fake_quant_fwd(x, d, z, bits, sym, codes=True)
        np.testing.assert_array_equal(host(y), g[t + "_y"], err_msg=t)
        _, qref = R.fake_quant(g[t + "_x"], host(d), host(z), bits, sym)
        cref = (qref.astype(np.int64) & 0xFF).astype(np.uint8)
        np.testing.assert_array_equal(codes.cpu().numpy(), cref, err_msg=t)
        # STE backward
        xr = x.clone().requires_grad_(True)
        dd = d.clone().requires_grad_(True)
        zz = z.clone().requires_grad_(True)
        yy = K.fake_quant(xr, dd, zz, bits, sym)
        yy.backward(dev(g[t + "_gy"]))
        np.testing.assert_array_equal(host(xr.grad), g[t + "_gx"], err_msg=t)
        close(host(dd.grad).reshape(-1), g[t + "_gdelta"], rtol=1e-4, atol=1e-4)
        close(host(zz.grad).reshape(-1), g[t + "_gzp"], rtol=1e-4, atol=1e-4)


def test_uaq_specials_golden(K, golden):
    """NaN / +-inf / +-0 / +-3e38 inputs against the reference (uaq_specials.npz): torch.clamp
    keeps NaN and round_ste turns an infinite x/delta into NaN, so the dequant is NaN there;
    every other output and gx bit for bit, the reductions within the usual tolerance (NaN
    where the reference's sum is NaN).  Per-tensor (float4 stream), per-channel (LDS tile
    kernel), the multi-tensor table, and ChannelQuantAct's torch.round q/dq."""
    g = golden("uaq_specials")
    for t in [k for k in tags(g, "_gdelta") if not k.startswith("act_")]:
        bits = int(t.split("_")[0][1:])
        sym = "_sym_" in t
        cw = "_cw_" in t
        x = g[t + "_x"]
        shape = (-1,) + (1,) * (x.ndim - 1) if cw else (1,)
        d, z = dev(g[t + "_delta"].reshape(shape)), dev(g[t + "_zp"].reshape(shape))
        y, _ = K.fake_quant_fwd(dev(x), d, z, bits, sym)
        np.testing.assert_array_equal(host(y), g[t + "_y"], err_msg=t)
        assert np.isnan(host(y)).sum() == np.isnan(g[t + "_y"]).sum() > np.isnan(x).sum(), t
        if cw:
            ym = K.fake_quant_multi([dev(x)], [d], [z], bits, sym)[0]
            np.testing.assert_array_equal(host(ym), g[t + "_y"], err_msg=t)
        xr, dd, zz = dev(x).requires_grad_(True), d.clone().requires_grad_(True), z.clone().requires_grad_(True)
        K.fake_quant(xr, dd, zz, bits, sym).backward(dev(g[t + "_gy"]))
        np.testing.assert_array_equal(host(xr.grad), g[t + "_gx"], err_msg=t)
        close(host(dd.grad).reshape(-1), g[t + "_gdelta"], rtol=1e-4, atol=1e-4)
        close(host(zz.grad).reshape(-1), g[t + "_gzp"], rtol=1e-4, atol=1e-4)
        np.testing.assert_array_equal(np.isnan(host(dd.grad).reshape(-1)), np.isnan(g[t + "_gdelta"]))
    x = g["b4_asym_pt_mse_x"]
    d, z = dev(g["b4_asym_pt_mse_delta"]), dev(g["b4_asym_pt_mse_zp"])
    for k in (0, 1):
        dd, zz = d.clone().requires_grad_(True), z.clone().requires_grad_(True)
        ya = K.round_quant(dev(x), dd, zz, 4, False, scale=float(g[f"act_s{k}_scale"][0]))
        np.testing.assert_array_equal(host(ya), g[f"act_s{k}_y"], err_msg=f"act_s{k}")
        ya.backward(dev(g["b4_asym_pt_mse_gy"]))
        close(host(dd.grad).reshape(-1), g[f"act_s{k}_gdelta"], rtol=1e-4, atol=1e-4)
        close(host(zz.grad).reshape(-1), g[f"act_s{k}_gzp"], rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("relu", [0, 1, 2])
def test_bias_act_quant_specials_vs_oracle(K, relu):
    """The fused epilogue's act q/dq (K13 + K1 in one pass, forward and the fused tail's
    recompute) on NaN / +-inf / huge pre-activations: the act quantizer's round_ste and
    torch.clamp semantics, bit for bit against the oracle applied to bias_act's output."""
    gen = torch.Generator().manual_seed(31 + relu)
    shape = (4, 8, 7, 7)
    y = torch.randn(shape, generator=gen).cuda() * 4
    y.view(-1)[:8] = torch.tensor([float("nan"), float("inf"), -float("inf"), 3e38, -3e38,
                                   -0.0, 0.0, 6.0])
    b = torch.randn(shape[1], generator=gen).cuda()
    d, z = torch.tensor([0.21]).cuda(), torch.tensor([3.0]).cuda()
    with torch.no_grad():
        a = K.bias_act_quant(y, b, None, relu, d, z, 4)
        pre = K.bias_act(y, b, None, relu)
    ref, _ = R.fake_quant(host(pre), np.float32(0.21), np.float32(3.0), 4)
    np.testing.assert_array_equal(host(a).view(np.int32), ref.view(np.int32))
    assert np.isnan(ref).any()


def test_uaq_zero_range(K, golden):
    g = golden("uaq")
    x = dev(g["zero_x"])
    d, z, _ = K.scale_init(x, 2, False, True, "max")
    np.testing.assert_array_equal(host(d).reshape(-1), g["zero_delta"])
    y, _ = K.fake_quant_fwd(x, d, z, 2)
    np.testing.assert_array_equal(host(y), g["zero_y"])


@pytest.mark.parametrize("shape,bits", [((512, 256, 3, 3), 2), ((64, 3, 7, 7), 8), ((1000, 512), 4),
                                        ((96, 1, 3, 3), 2)])
def test_scale_init_vs_oracle(K, shape, bits):
    gen = torch.Generator().manual_seed(1005)
    w = torch.randn(shape, generator=gen) * 0.05
    x = w.cuda()
    for method in ("max", "mse"):
        d, z, r = K.scale_init(x, bits, False, True, method)
        rd, rz, rr = R.init_scale(w.numpy(), bits, False, True, method)
        hd, hz = host(d).reshape(-1), host(z).reshape(-1)
        if method == "max":
            np.testing.assert_array_equal(hd, rd.reshape(-1))
            np.testing.assert_array_equal(hz, rz.reshape(-1))
        else:
            # first-strict-min over Lp(2.4) scores: a flip is only allowed where the two
            # candidates' scores agree to 1e-5 relative (summation order / pow ulp)
            flips = np.nonzero((hd != rd.reshape(-1)) | (hz != rz.reshape(-1)))[0]
            assert len(flips) <= max(1, shape[0] // 200), f"{len(flips)} channel flips"


def test_scale_init_per_tensor_mse(K):
    gen = torch.Generator().manual_seed(7)
    x = torch.relu(torch.randn(8, 64, 28, 28, generator=gen))
    d, z, r = K.scale_init(x.cuda(), 4, False, False, "mse")
    rd, rz, rr = R.init_scale(x.numpy(), 4, False, False, "mse")
    assert host(d) == rd and host(z) == rz and host(r) == rr


def test_scale_init_specials_golden(K, golden):
    """NaN / +-inf / 3e38 / constant / zero rows planted BEFORE the init
    (make_golden.gen_init_specials, the reference's init_quantization_scale,
    quant_layer.py:100-166).  Where the reference returns a usable scale ssq_scale_init's is
    bit-identical (delta = inf for a +inf row included); where the reference raises or returns
    None, K.scale_init raises ScaleInitError -- and with check=False the NaN-marked rows are
    exactly the planted row (3; per-tensor: the one row)."""
    d = golden("init_specials")
    n_raise = 0
    for tag in d["cases"]:
        tag = str(tag)
        method, cw, sym = tag.split("_")[:3]
        cw, sym = cw == "cw", sym == "sym"
        x = dev(d[tag + "_x"])
        status = int(d[tag + "_status"][0])
        if status != 0:
            with pytest.raises(K.ScaleInitError):
                K.scale_init(x, 4, sym, cw, method)
            dl, zp, _ = K.scale_init(x, 4, sym, cw, method, check=False)
            bad = (torch.isnan(dl) | torch.isnan(zp)).flatten().nonzero().flatten().tolist()
            assert bad == ([3] if cw else [0]), (tag, bad)
            n_raise += 1
            continue
        dl, zp, rz = K.scale_init(x, 4, sym, cw, method)
        np.testing.assert_array_equal(host(dl).ravel(), d[tag + "_delta"], err_msg=tag)
        np.testing.assert_array_equal(host(zp).ravel(), d[tag + "_zp"], err_msg=tag)
        np.testing.assert_array_equal(host(rz).ravel(), d[tag + "_rawzp"], err_msg=tag)
    assert n_raise == sum(int(d[str(t) + "_status"][0]) != 0 for t in d["cases"]) > 10


@pytest.mark.parametrize("n", [0, 1, 3, 4, 5, 1023, 4097, 1 << 20])
def test_fq_ragged_sizes(K, n):
    gen = torch.Generator().manual_seed(n)
    x = torch.randn(max(n, 1), generator=gen)[:n]
    d, z = torch.tensor(0.05), torch.tensor(3.0)
    y, c = K.fake_quant_fwd(x.cuda(), d.cuda(), z.cuda(), 3, codes=True)
    ry, rq = R.fake_quant(x.numpy(), d.numpy(), z.numpy(), 3)
    np.testing.assert_array_equal(host(y), ry)
    np.testing.assert_array_equal(c.cpu().numpy(), rq.astype(np.uint8))


@pytest.mark.parametrize("variant", [1 | (256 << 8), 1 | (3 << 4) | (512 << 8),
                                     (2 << 4) | (64 << 8) | (1 << 24), 3 | (4 << 4) | (128 << 8)])
def test_fq_streaming_variants(K, variant):
    """Every launch-geometry variant of the per-tensor kernel is bit-exact, including
    sizes that end mid-step and inside the scalar tail."""
    old = K.set_variant(variant)
    try:
        for n in (4, 1020, 65536 * 4 + 12, 256 * 256 * 4 * 9 + 3, 3 << 20):
            gen = torch.Generator().manual_seed(n)
            x = torch.randn(n, generator=gen)
            d, z = torch.tensor(0.11), torch.tensor(7.0)
            y, c = K.fake_quant_fwd(x.cuda(), d.cuda(), z.cuda(), 4, codes=True)
            ry, rq = R.fake_quant(x.numpy(), d.numpy(), z.numpy(), 4)
            np.testing.assert_array_equal(host(y), ry)
            np.testing.assert_array_equal(c.cpu().numpy(), rq.astype(np.uint8))
    finally:
        K.set_variant(old)


def _boundary_inputs(d, n_per=4096, seed=5):
    """Values x whose quotient x/d lands on or one ulp either side of the rounding
    boundaries k+0.5 (rint) and k (floor), plus zeros, subnormals and huge values."""
    gen = np.random.default_rng(seed)
    k = gen.integers(-300, 300, n_per).astype(np.float32)
    base = np.concatenate([(k + np.float32(0.5)) * np.float32(d), k * np.float32(d)]).astype(np.float32)
    xs = [base, np.nextafter(base, np.float32(np.inf)), np.nextafter(base, np.float32(-np.inf)),
          np.array([0.0, -0.0, 1e-45, -1e-45, 1e-40, -3e-39, 1e30, -1e30, 3e38], np.float32),
          (gen.standard_normal(n_per) * 10).astype(np.float32)]
    x = np.concatenate(xs).astype(np.float32)
    return x[: len(x) // 4 * 4]


@pytest.mark.parametrize("rcp", [0, 1])
@pytest.mark.parametrize("d", [0.05, 0.3, 1e-8, 7.0e-3, 2.0 ** -70, 3.0e20])
def test_fq_rounding_boundaries(K, d, rcp):
    """Quotients on / one ulp beside the rint and floor boundaries, zeros, subnormals,
    huge values: codes and dequantized values bit-exact against the oracle, with the IEEE
    divide and with the reciprocal-form fast path (variant bit 27)."""
    x = torch.from_numpy(_boundary_inputs(d))
    dd, z = torch.tensor(np.float32(d)), torch.tensor(2.0)
    old = K.set_variant(1 | (3 << 4) | (256 << 8) | (rcp << 27))
    try:
        a, ca = K.fake_quant_fwd(x.cuda(), dd.cuda(), z.cuda(), 8, codes=True)
        # a large ReLU-like tensor: whole waves take the fast path when rcp is on
        big = torch.relu(torch.randn(1 << 22, generator=torch.Generator().manual_seed(9))) * float(d)
        b, cb = K.fake_quant_fwd(big.cuda(), dd.cuda(), z.cuda(), 8, codes=True)
    finally:
        K.set_variant(old)
    ry, rq = R.fake_quant(x.numpy(), dd.numpy(), z.numpy(), 8)
    np.testing.assert_array_equal(host(a).view(np.int32), ry.view(np.int32))
    np.testing.assert_array_equal(ca.cpu().numpy(), rq.astype(np.uint8))
    ry, rq = R.fake_quant(big.numpy(), dd.numpy(), z.numpy(), 8)
    np.testing.assert_array_equal(host(b).view(np.int32), ry.view(np.int32))
    np.testing.assert_array_equal(cb.cpu().numpy(), rq.astype(np.uint8))


def test_fq_per_channel_unaligned(K):
    # conv1-like rows of 147 elements: float4 vectors straddle channel boundaries
    gen = torch.Generator().manual_seed(3)
    w = torch.randn(64, 3, 7, 7, generator=gen) * 0.1
    d, z, _ = R.init_scale(w.numpy(), 8, False, True, "max")
    y, _ = K.fake_quant_fwd(w.cuda(), dev(d), dev(z), 8)
    np.testing.assert_array_equal(host(y), R.fake_quant(w.numpy(), d, z, 8)[0])
    # and through an offset (non 16-B aligned) view
    big = torch.randn(1 + w.numel(), generator=gen).cuda()
    view = big[1:].view(w.shape)
    y2, _ = K.fake_quant_fwd(view, dev(d), dev(z), 8)
    np.testing.assert_array_equal(host(y2), R.fake_quant(host(view), d, z, 8)[0])


@pytest.mark.parametrize("shape", [(96, 2048, 3, 3), (1024, 512, 3, 3), (50, 65, 2, 2),
                                   (1000, 512)])
def test_fq_per_channel_long_rows(K, shape):
    """Per-channel q/dq with rows of >= 256 elements (fq_fwd_rows: wave-uniform channel
    parameters, waves spanning two rows), with codes: bit-exact against the oracle."""
    gen = torch.Generator().manual_seed(sum(shape))
    x = torch.randn(shape, generator=gen) * 0.05
    d, z, _ = R.init_scale(x.numpy(), 2, False, True, "max")
    y, c = K.fake_quant_fwd(x.cuda(), dev(d), dev(z), 2, codes=True)
    ry, rq = R.fake_quant(x.numpy(), d, z, 2)
    np.testing.assert_array_equal(host(y).view(np.int32), ry.view(np.int32))
    np.testing.assert_array_equal(c.cpu().numpy().ravel(), rq.astype(np.uint8).ravel())


def test_fq_multi_segment(K):
    gen = torch.Generator().manual_seed(11)
    shapes = [(64, 3, 7, 7), (64, 64, 3, 3), (128, 64, 1, 1), (1000, 512), (8, 1, 3, 3)]
    ws = [torch.randn(s, generator=gen) * 0.05 for s in shapes]
    params = [R.init_scale(w.numpy(), 2, False, True, "max") for w in ws]
    ys = K.fake_quant_multi([w.cuda() for w in ws], [dev(p[0]) for p in params],
                            [dev(p[1]) for p in params], 2)
    for w, p, y in zip(ws, params, ys):
        np.testing.assert_array_equal(host(y), R.fake_quant(w.numpy(), p[0], p[1], 2)[0])
    # caller-owned outputs (out=): written in place, same bits; wrong shapes refused
    outs = [torch.full(s, float("nan"), device="cuda") for s in shapes]
    ys2 = K.fake_quant_multi([w.cuda() for w in ws], [dev(p[0]) for p in params],
                             [dev(p[1]) for p in params], 2, out=outs)
    for y, y2, o in zip(ys, ys2, outs):
        assert y2 is o
        np.testing.assert_array_equal(host(y2), host(y))
    with pytest.raises(ValueError):
        K.fake_quant_multi([w.cuda() for w in ws], [dev(p[0]) for p in params],
                           [dev(p[1]) for p in params], 2, out=outs[::-1])
    # a launch plan: the same bits every launch, in-place input updates seen, riding on a
    # per-tensor launch under deferred_fq_multi
    xs = [w.cuda() for w in ws]
    plan = K.FqMultiPlan(xs, [dev(p[0]) for p in params], [dev(p[1]) for p in params], 2)
    for y, y3 in zip(ys, plan()):
        np.testing.assert_array_equal(host(y3), host(y))
    xs[1].mul_(-1.0)
    act = torch.randn(4, 8, 7, 7, generator=gen).relu_().cuda()
    with K.deferred_fq_multi():
        ys4 = plan()
        K.fake_quant_fwd(act, dev([0.1]), dev([0.0]), 4)
    np.testing.assert_array_equal(host(ys4[1]), R.fake_quant(-ws[1].numpy(), params[1][0],
                                                            params[1][1], 2)[0])
    np.testing.assert_array_equal(host(ys4[0]), host(ys[0]))


def test_fq_multi_many_ragged_segments(K):
    """More segments than one launch holds (ResNet-50 has 54 layers), rows of 1-3 and
    odd lengths (float4s straddling channels), an unaligned view, tiles crossing rows."""
    gen = torch.Generator().manual_seed(12)
    shapes = []
    for i in range(61):
        shapes.append([(7, 1), (5, 2), (9, 3), (33, 3, 7, 7), (16, 5, 1, 1), (1000, 512),
                       (64, 64, 3, 3), (3, 4099)][i % 8])
    ws = [torch.randn(s, generator=gen) * 0.05 for s in shapes]
    params = [R.init_scale(w.numpy(), 4, False, True, "max") for w in ws]
    xs = [w.cuda() for w in ws]
    big = torch.randn(1 + ws[5].numel(), generator=gen).cuda()
    xs[5] = big[1:].view(ws[5].shape)           # not 16-B aligned -> scalar path
    ys = K.fake_quant_multi(xs, [dev(p[0]) for p in params], [dev(p[1]) for p in params], 4)
    for x, p, y in zip(xs, params, ys):
        np.testing.assert_array_equal(host(y), R.fake_quant(host(x), p[0], p[1], 4)[0])


# ------------------------------------------------------------------ K5-K9 on goldens
def _cq(g, tag):
    w = g[tag + "_w"]
    is_fc = w.ndim != 4
    shape = (-1, 1) if is_fc else (-1, 1, 1, 1)
    return w, is_fc, g[tag + "_delta"].reshape(shape), g[tag + "_zp"].reshape(shape), int(tag.rsplit("_b", 1)[1])


CQ_TAGS = ["conv_b2", "conv_b4", "fc_b2", "fc_b4", "dw_b2", "dw_b4"]
# channelquant_specials: the same cases with NaN / +-inf / +-0 / +-3e38 planted into W after
# the scale init (make_golden.SPECIALS): NaN wherever the reference gives NaN, the rest as
# before (assert_array_equal / assert_allclose compare NaN positions as equal)
CQ_FILES = ["channelquant", "channelquant_specials"]


@pytest.mark.parametrize("fname", CQ_FILES)
@pytest.mark.parametrize("tag", CQ_TAGS)
def test_shift_init_golden(K, golden, tag, fname):
    g = golden(fname)
    w, is_fc, d, z, bits = _cq(g, tag)
    alpha, beta, _ = K.shift_init(dev(w), dev(d), SHIFTS)
    close(host(alpha), g[tag + "_alpha0"], rtol=1e-5, atol=1e-6)
    close(host(beta), g[tag + "_beta"], rtol=1e-5, atol=1e-5)
    np.testing.assert_array_equal(host(beta) >= 0, g[tag + "_beta"] >= 0)


@pytest.mark.parametrize("fname", CQ_FILES)
@pytest.mark.parametrize("tag", CQ_TAGS)
def test_adashift_golden(K, golden, tag, fname):
    g = golden(fname)
    w, is_fc, d, z, bits = _cq(g, tag)
    alpha, beta = g[tag + "_alpha"], g[tag + "_beta"]
    np.testing.assert_array_equal(host(K.get_delta(dev(d), dev(alpha), SHIFTS, w.shape)),
                                  g[tag + "_delta_sel"])
    for ht, hr in ((0, 0), (1, 1), (0, 1), (1, 0)):
        k = f"{tag}_t{ht}r{hr}"
        a = dev(alpha).requires_grad_(True)
        b = dev(beta).requires_grad_(True)
        y = K.adashift(a, b, dev(w), dev(d), dev(z), SHIFTS, bits, False, ht, hr)
        if ht and hr:
            np.testing.assert_array_equal(host(y), g[k + "_y"], err_msg=k)
        else:
            close(host(y), g[k + "_y"], rtol=1e-5, atol=1e-7)
        if not ht:
            y.backward(dev(g[tag + "_gy"]))
            close(host(a.grad), g[k + "_galpha"], rtol=1e-4, atol=1e-6)
            if not hr:
                close(host(b.grad), g[k + "_gbeta"], rtol=1e-4, atol=1e-7)
    y, codes = K.adashift_codes(dev(alpha), dev(beta), dev(w), dev(d), dev(z), SHIFTS, bits, False)
    np.testing.assert_array_equal(host(y), g[tag + "_t1r1_y"])
    c = codes.cpu().numpy().astype(np.float32)
    ref = g[tag + "_t1r1_y"]
    ok = ~np.isnan(ref)                 # a NaN weight has no integer code
    np.testing.assert_array_equal(((c - z) * d)[ok], ref[ok])   # What = (q - zp) * delta


@pytest.mark.parametrize("fname", CQ_FILES)
@pytest.mark.parametrize("tag", CQ_TAGS)
def test_lhs_adaround_golden(K, golden, tag, fname):
    g = golden(fname)
    w, is_fc, d, z, bits = _cq(g, tag)
    alpha = g[tag + "_lhs_alpha"]
    a = dev(alpha).requires_grad_(True)
    y = K.lhs(a, dev(w), dev(d), dev(z), SHIFTS, bits, False, False)
    close(host(y), g[tag + "_lhs_t0_y"], atol=1e-7)
    y.backward(dev(g[tag + "_gy"]))
    close(host(a.grad), g[tag + "_lhs_t0_galpha"], rtol=1e-4, atol=1e-6)
    y = K.lhs(dev(alpha), dev(w), dev(d), dev(z), SHIFTS, bits, False, True)
    np.testing.assert_array_equal(host(y), g[tag + "_lhs_t1_y"])
    dsel = K.get_delta(dev(d), dev(alpha), SHIFTS, w.shape)
    np.testing.assert_array_equal(host(dsel), g[tag + "_ar_delta"])
    close(host(K.rect_init(dev(w), dsel)), g[tag + "_ar_beta0"], atol=1e-5)
    beta = g[tag + "_ar_beta"]
    y = K.adaround(dev(beta), dev(w), dsel, dev(z), bits, False, True)
    np.testing.assert_array_equal(host(y), g[tag + "_ar_r1_y"])
    b = dev(beta).requires_grad_(True)
    y = K.adaround(b, dev(w), dsel, dev(z), bits, False, False)
    close(host(y), g[tag + "_ar_r0_y"], atol=1e-7)
    y.backward(dev(g[tag + "_gy"]))
    close(host(b.grad), g[tag + "_ar_r0_gbeta"], rtol=1e-4, atol=1e-7)


@pytest.mark.parametrize("fname", ["adaround", "adaround_specials"])
@pytest.mark.parametrize("name", ["conv", "fc"])
def test_adaround_quantizer_golden(K, golden, name, fname):
    g = golden(fname)
    w = g[name + "_w"]
    shape = (-1, 1) if w.ndim == 2 else (-1, 1, 1, 1)
    d, z = g[name + "_delta"].reshape(shape), g[name + "_zp"].reshape(shape)
    close(host(K.rect_init(dev(w), dev(d))), g[name + "_alpha0"], atol=1e-5)
    a = g[name + "_alpha"]
    np.testing.assert_array_equal(host(K.adaround(dev(a), dev(w), dev(d), dev(z), 2, False, True)),
                                  g[name + "_s0_y"])
    ar = dev(a).requires_grad_(True)
    y = K.adaround(ar, dev(w), dev(d), dev(z), 2, False, False)
    close(host(y), g[name + "_s1_y"], atol=1e-7)
    y.backward(dev(g[name + "_gy"]))
    close(host(ar.grad), g[name + "_s1_galpha"], rtol=1e-4, atol=1e-7)


def test_adashift_large_vs_oracle(K):
    """ResNet-18 layer4 conv shape: hard codes bit-exact, soft within 1e-5."""
    gen = torch.Generator().manual_seed(1005)
    w = (torch.randn(512, 512, 3, 3, generator=gen) * 0.02).numpy()
    d, z, _ = R.init_scale(w, 2, False, True, "max")
    xq, alpha, beta = R.init_v_beta(w, d, SHIFTS)
    a, b, _ = K.shift_init(dev(w), dev(d), SHIFTS)
    close(host(a), alpha, atol=1e-6)
    np.testing.assert_array_equal(host(b) >= 0, beta >= 0)
    y = K.adashift(dev(alpha), dev(beta), dev(w), dev(d), dev(z), SHIFTS, 2, False, True, True)
    np.testing.assert_array_equal(host(y), R.adashift_fwd(xq, alpha, beta, d, z, 2, False, False, True, True))
    y = K.adashift(dev(alpha), dev(beta), dev(w), dev(d), dev(z), SHIFTS, 2, False, False, False)
    close(host(y), R.adashift_fwd(xq, alpha, beta, d, z, 2, False, False, False, False), atol=1e-7)


# ------------------------------------------------------------------ K10-K12
def test_inpscale_golden(K, golden):
    g = golden("inpscale")
    for bits in (2, 4):
        w = g[f"b{bits}_w"]
        d = g[f"b{bits}_delta"].reshape(-1, 1, 1, 1)
        rz = g[f"b{bits}_rawzp"].reshape(-1, 1, 1, 1)
        for level in (1, 2, 8, 64):
            for thr in (1, 2):
                t = f"b{bits}_l{level}_t{thr}"
                inp = K.inpscale_search(dev(w), dev(d), dev(rz), bits, level, float(thr))
                np.testing.assert_array_equal(host(inp), g[t + "_inp"], err_msg=t)
                np.testing.assert_array_equal(host(K.inpscale_fwd(dev(w), inp, dev(d), dev(rz), bits)),
                                              g[t + "_y"], err_msg=t)


def test_lp_loss_golden(K, golden):
    g = golden("loss")
    for p in (1.0, 2.0, 2.4):
        for red in ("none", "all"):
            pr = dev(g["pred"]).requires_grad_(True)
            loss = K.lp_loss(pr, dev(g["tgt"]), p, red)
            loss.backward()
            close(loss.item(), g[f"p{p}_{red}_loss"][0], rtol=1e-5)
            if p == 2.0:
                np.testing.assert_array_equal(host(pr.grad), g[f"p{p}_{red}_grad"])
            else:
                close(host(pr.grad), g[f"p{p}_{red}_grad"], rtol=1e-5, atol=1e-9)
            l2, gr = K.lp_loss_and_grad(dev(g["pred"]), dev(g["tgt"]), p, red)
            close(host(l2)[0], g[f"p{p}_{red}_loss"][0], rtol=1e-5)
            close(host(gr), g[f"p{p}_{red}_grad"], rtol=1e-5, atol=1e-9)


def test_regularizers_golden(K, golden):
    g = golden("loss")
    for b in (0.0, 20.0, 11.3, 2.0):
        a = dev(g["reg_alpha"]).requires_grad_(True)
        l = K.shift_reg(a, 0.1, b, 0)
        l.backward()
        close(l.item(), g[f"regS_b{b}_loss"][0], rtol=1e-5)
        close(host(a.grad), g[f"regS_b{b}_grad"], rtol=1e-4, atol=1e-7)
        v = dev(g["reg_beta"]).requires_grad_(True)
        l = K.round_reg(v, 0.01, b)
        l.backward()
        close(l.item(), g[f"regR_b{b}_loss"][0], rtol=1e-5)
        close(host(v.grad), g[f"regR_b{b}_grad"], rtol=1e-4, atol=1e-7)
    a = dev(g["reg_alpha"]).requires_grad_(True)
    l = K.shift_reg(a, 0.1, 0.0, 1)
    l.backward()
    close(l.item(), g["regE_loss"][0], rtol=1e-5)
    close(host(a.grad), g["regE_grad"], rtol=1e-4, atol=1e-7)


def test_gather_rows(K):
    gen = torch.Generator().manual_seed(5)
    a = torch.randn(64, 16, 7, 7, generator=gen)
    b = torch.randn(64, 8, 5, 3, generator=gen)
    idx = torch.randperm(64, generator=gen)[:32]
    ga, gb = K.gather_rows2(a.cuda(), idx, b.cuda())
    np.testing.assert_array_equal(host(ga), a[idx].numpy())
    np.testing.assert_array_equal(host(gb), b[idx].numpy())


def test_fused_bwd_with_reg_matches_separate(K, golden):
    """adaShift backward with the fused shift regulariser == separate reg gradient."""
    g = golden("channelquant")
    w, is_fc, d, z, bits = _cq(g, "conv_b2")
    alpha, beta = g["conv_b2_alpha"], g["conv_b2_beta"]
    gy = dev(g["conv_b2_gy"])
    a1 = dev(alpha).requires_grad_(True)
    y = K.adashift(a1, dev(beta), dev(w), dev(d), dev(z), SHIFTS, bits, False, False, False)
    (y * gy).sum().backward()
    a2 = dev(alpha).requires_grad_(True)
    K.shift_reg(a2, 0.1, 11.3, 0).backward()
    a3 = dev(alpha).requires_grad_(True)
    vals = torch.empty(alpha.shape[0], device="cuda")
    y = K.adashift(a3, dev(beta), dev(w), dev(d), dev(z), SHIFTS, bits, False, False, False,
                   reg=(0.1, 11.3, vals, None))
    (y * gy).sum().backward()
    close(host(a3.grad), host(a1.grad) + host(a2.grad), rtol=1e-5, atol=1e-7)
    # device-side (lambda, b) form used under HIP-graph capture
    a4 = dev(alpha).requires_grad_(True)
    regp = torch.tensor([0.1, 11.3], device="cuda")
    y = K.adashift(a4, dev(beta), dev(w), dev(d), dev(z), SHIFTS, bits, False, False, False,
                   reg=(0.0, 0.0, vals, regp))
    (y * gy).sum().backward()
    close(host(a4.grad), host(a3.grad), rtol=1e-6, atol=1e-9)
    a3 = dev(alpha).requires_grad_(True)
    y = K.adashift(a3, dev(beta), dev(w), dev(d), dev(z), SHIFTS, bits, False, False, False,
                   reg=(0.1, 11.3, vals, None))
    (y * gy).sum().backward()
    close(host(a3.grad), host(a1.grad) + host(a2.grad), rtol=1e-5, atol=1e-7)


def _act_ref(t, relu):
    """The eager activation of an activation code (0 identity, 1 ReLU, 2 ReLU6)."""
    return torch.nn.functional.relu6(t) if relu == 2 else torch.relu(t) if relu else t


# activation edge values: signed zeros, NaN, the ReLU6 clamp edge and its neighbours, inf
EDGE = [-0.0, float("nan"), 0.0, 6.0, 6.0000005, 5.9999995, float("inf"), -float("inf")]


@pytest.mark.parametrize("shape,res,relu", [((4, 8, 7, 7), True, True), ((3, 5, 6, 6), False, True),
                                            ((2, 16, 14, 14), True, False), ((2, 3, 5, 3), False, False),
                                            ((32, 64, 56, 56), True, True), ((4, 8, 7, 7), True, 2),
                                            ((2, 3, 5, 3), False, 2), ((32, 64, 56, 56), False, 2),
                                            ((48, 64, 56, 56), True, True)])  # > 1 grid trip
def test_bias_act_matches_eager_ops(K, shape, res, relu):
    """K13 epilogue == (y + bias) (+ residual) -> ReLU / ReLU6 as separate fp32 torch ops
    on the device, bit for bit (-0.0 / NaN / the clamp edges through the activation), and
    its backward."""
    gen = torch.Generator().manual_seed(sum(shape))
    y = torch.randn(shape, generator=gen).cuda()
    y.view(-1)[:8] = torch.tensor(EDGE)
    b = torch.randn(shape[1], generator=gen).cuda()
    b[0] = 0.0
    r = torch.randn(shape, generator=gen).cuda() if res else None
    if res:
        r.view(-1)[:8] = 0.0
    ref = y + b.view(1, -1, 1, 1)
    if res:
        ref = ref + r
    ref = _act_ref(ref, relu)
    out = K.bias_act(y, b, r, relu)
    np.testing.assert_array_equal(host(out).view(np.int32), host(ref).view(np.int32))
    # backward against autograd of the eager ops
    yr = y.clone().requires_grad_(True)
    rr = r.clone().requires_grad_(True) if res else None
    o = K.bias_act(yr, b, rr, relu)
    g = torch.randn(shape, generator=gen).cuda()
    o.backward(g)
    ye = y.clone().requires_grad_(True)
    re_ = r.clone().requires_grad_(True) if res else None
    e = ye + b.view(1, -1, 1, 1)
    if res:
        e = e + re_
    e = _act_ref(e, relu)
    e.backward(g)
    np.testing.assert_array_equal(host(yr.grad), host(ye.grad))
    if res:
        np.testing.assert_array_equal(host(rr.grad), host(re_.grad))


@pytest.mark.parametrize("affine", [False, True])
@pytest.mark.parametrize("act", [False, True])
def test_quant_block_fused_epilogue_matches_unfused(K, act, affine):
    """A QuantBasicBlock forward/backward through the fused epilogue equals the eager
    path (fusion disabled) bit for bit; with act quant on, the act q/dq runs inside the
    epilogue pass and the act-delta gradients match too."""
    from shiftedscalequantization_amd import nets, quant as Q
    torch.manual_seed(3)
    ds = torch.nn.Sequential(torch.nn.Conv2d(16, 32, 1, stride=2, bias=False), torch.nn.BatchNorm2d(32))
    blk = nets.BasicBlock(16, 32, stride=2, downsample=ds).eval()
    qnn = Q.QuantModel(torch.nn.Sequential(blk), {"n_bits": 4, "channel_wise": True, "scale_method": "max"},
                       {"n_bits": 8, "channel_wise": False, "scale_method": "max"}).cuda()
    qb = qnn.model[0]
    qnn.set_quant_state(True, act)
    x = torch.randn(4, 16, 14, 14).cuda()
    with torch.no_grad():
        qnn(x)                                       # init the quantizers
    _compare_fused_unfused(qb, x, act, _set_affine(qb) if affine else ())


@pytest.mark.parametrize("affine", [False, True])
@pytest.mark.parametrize("act", [False, True])
def test_epilogue_into_gemm_bit_identical(K, act, affine):
    """kernels.EPI_INTO_GEMM: a BasicBlock on ResNet-18 layer3's small plane (256 -> 256,
    14x14: conv2's forward and weight gradient are im2col GEMMs) folds conv1's K13 epilogue
    into conv2's im2col build (ssq_gemm_col_epilogue; no epilogue forward launch, no
    activation written).  Output, input gradient, both conv weights' gradients, gamma^z /
    phi^z and act-delta gradients equal the unfolded path's bit for bit."""
    from shiftedscalequantization_amd import nets, quant as Q
    torch.manual_seed(5)
    blk = nets.BasicBlock(256, 256, stride=1).eval()
    qnn = Q.QuantModel(torch.nn.Sequential(blk), {"n_bits": 2, "channel_wise": True, "scale_method": "max"},
                       {"n_bits": 4, "channel_wise": False, "scale_method": "max"}).cuda()
    qb = qnn.model[0]
    qnn.set_quant_state(True, act)
    x = torch.randn(32, 256, 14, 14).cuda()    # the recon loop's batch (its GEMM shapes)
    with torch.no_grad():
        qnn(x)
    ps = _set_affine(qb) if affine else []
    ws = [qb.conv1.weight, qb.conv2.weight]
    calls, orig = [], K.epi_conv_gemm

    def spy(*a, **k):
        calls.append(1)
        return orig(*a, **k)

    outs = []
    prev, det = K.EPI_INTO_GEMM, torch.backends.cudnn.deterministic
    K.epi_conv_gemm = spy
    torch.backends.cudnn.deterministic = True      # MIOpen's input gradients run to run
    try:
        for fold in (False, True, False):
            K.EPI_INTO_GEMM = fold
            for t in ws + list(ps) + list(_act_deltas(qb)):
                t.grad = None
            xx = x.clone().requires_grad_(True)
            y = qb(xx)
            gy = torch.linspace(-1, 1, y.numel(), device=y.device).view_as(y)
            y.backward(gy)
            outs.append([host(y), host(xx.grad)] + [host(t.grad) for t in ws + list(ps)] +
                        ([host(d.grad) for d in _act_deltas(qb)] if act else []))
            if fold:
                n_fold = len(calls)
                calls.clear()
    finally:
        K.EPI_INTO_GEMM, K.epi_conv_gemm = prev, orig
        torch.backends.cudnn.deterministic = det
    # folded wherever the act quantizer allows it (not act-quant without the affine form)
    assert n_fold == (0 if (act and not affine) else 1) and not calls
    assert len(outs[0]) == len(outs[1]) == len(outs[2])
    for a, b in zip(outs[0], outs[2]):     # the unfolded path is itself run-to-run identical
        np.testing.assert_array_equal(a.view(np.int32), b.view(np.int32))
    for a, b in zip(outs[1], outs[0]):
        np.testing.assert_array_equal(a.view(np.int32), b.view(np.int32))


def _act_deltas(qb):
    from shiftedscalequantization_amd import quant as Q
    ds = [qb.act_quantizer.delta]
    ds += [m.act_quantizer.delta for m in qb.modules()
           if isinstance(m, Q.QuantModule) and not m.disable_act_quant]
    return [d for d in ds if d is not None]


def _set_affine(qb):
    """Random learned gamma^z / phi^z on every QuantModule of the block (--bias_cal)."""
    from shiftedscalequantization_amd import quant as Q
    gen = torch.Generator().manual_seed(77)
    ps = []
    for m in qb.modules():
        if isinstance(m, Q.QuantModule):
            c = m.alpha_out.numel()
            m.alpha_out.data = (1 + 0.1 * torch.randn(c, generator=gen)).view_as(m.alpha_out).cuda()
            m.beta_out.data = (0.1 * torch.randn(c, generator=gen)).view_as(m.beta_out).cuda()
            m.alpha_out.requires_grad_(True)
            m.beta_out.requires_grad_(True)
            ps += [m.alpha_out, m.beta_out]
    return ps


def _compare_fused_unfused(qb, x, act, affine=()):
    # under the reference's cudnn.deterministic (as the folded-epilogue test: run-to-run
    # identical input gradients).  The forward's values still differ between box types, and
    # the affine act-delta bound below is cancellation-sensitive to them (r5ev5 and r5ev7b,
    # this mode included: 3.6e-3 off on ~18 where other boxes stay inside 2.8e-3)
    det = torch.backends.cudnn.deterministic
    torch.backends.cudnn.deterministic = True
    try:
        _compare_fused_unfused_det(qb, x, act, affine)
    finally:
        torch.backends.cudnn.deterministic = det


def _compare_fused_unfused_det(qb, x, act, affine=()):
    from shiftedscalequantization_amd import quant as Q
    outs = []
    g = torch.randn(1, generator=torch.Generator().manual_seed(1))
    for fuse in (True, False):
        if not fuse:
            for m in qb.modules():
                if isinstance(m, Q.QuantModule):
                    m.epilogue_fusable = lambda inp: False
        for d in list(_act_deltas(qb)) + list(affine):
            d.grad = None
        xx = x.clone().requires_grad_(True)
        y = qb(xx)
        gy = torch.linspace(-1, 1, y.numel(), device=y.device).view_as(y) + g.item()
        y.backward(gy)
        outs.append((host(y), host(xx.grad), [host(d.grad) for d in _act_deltas(qb)] if act else [],
                     [host(p.grad) for p in affine]))
    np.testing.assert_array_equal(outs[0][0], outs[1][0])
    np.testing.assert_array_equal(outs[0][1], outs[1][1])
    assert len(outs[0][2]) == len(outs[1][2])
    for a, b in zip(outs[0][2], outs[1][2]):
        # the fused epilogue reduces the act-delta sums per (n, c) row (with or without
        # gamma^z / phi^z since r6), the fq backward per workgroup: the same fp32 terms --
        # (x/d)/d with two IEEE divides on both sides, as torch's div backward -- summed in
        # double in two orders.  Until r6 the float4 fq backward took (x/d)*(1/d), one ulp
        # per term of two ~1e2 sums that cancel to ~1e-2, and that ulp reached 2.0e-4 of the
        # result (r5ev5, r5ev7b: 18.1153 vs 18.1189).  Now only the double sums' order
        # differs: ~1e-16 * 1e4 of the result, far below one fp32 ulp
        np.testing.assert_allclose(a, b, rtol=1e-6, atol=0)
    for a, b in zip(outs[0][3], outs[1][3]):   # gamma / phi: double vs torch's fp32 sums
        np.testing.assert_allclose(a, b, rtol=1e-4, atol=1e-4 * np.abs(b).max())


@pytest.mark.parametrize("affine", [False, True])
@pytest.mark.parametrize("act", [False, True])
@pytest.mark.parametrize("kind", ["bottleneck", "resbottleneck", "inverted"])
def test_other_blocks_fused_epilogue_matches_unfused(K, kind, act, affine):
    """ResNet-50 / RegNetX / MobileNetV2 blocks: the fused conv-bias + residual (+ReLU)
    tail equals the eager ops bit for bit, forward and backward."""
    import torch.nn as nn
    from shiftedscalequantization_amd import nets, quant as Q
    torch.manual_seed(5)
    if kind == "bottleneck":
        ds = nn.Sequential(nn.Conv2d(32, 64, 1, stride=2, bias=False), nn.BatchNorm2d(64))
        blk, cin = nets.Bottleneck(32, 16, stride=2, downsample=ds), 32
    elif kind == "resbottleneck":
        blk, cin = nets.ResBottleneckBlock(32, 96, 2, 48), 32
    else:
        blk, cin = nets.InvertedResidual(24, 24, 1, 6), 24
    qnn = Q.QuantModel(nn.Sequential(blk.eval()), {"n_bits": 4, "channel_wise": True, "scale_method": "max"},
                       {"n_bits": 8, "channel_wise": False, "scale_method": "max"}).cuda()
    qb = qnn.model[0]
    assert isinstance(qb, Q.BaseQuantBlock)
    qnn.set_quant_state(True, act)
    x = torch.randn(4, cin, 14, 14).cuda()
    with torch.no_grad():
        qnn(x)
    if kind == "inverted":   # the ReLU6 layers take the fused epilogue (activation code 2)
        assert [m.act_code() for m in qb.conv] == [2, 2, 0]
        assert all(m.epilogue_fusable(x) for m in qb.conv)
    _compare_fused_unfused(qb, x, act, _set_affine(qb) if affine else ())


@pytest.mark.parametrize("shape", [(4, 8, 7, 7), (2, 3, 5, 3), (32, 64, 56, 56)])
@pytest.mark.parametrize("res", [False, True])
@pytest.mark.parametrize("relu", [0, 1, 2])
def test_bias_act_quant_matches_composed(K, shape, res, relu):
    """K13 + act q/dq in one pass == bias_act then fake_quant, bit for bit: the output,
    and the gradients of y, the residual, delta and zero_point (ReLU / ReLU6 backward
    folded into the STE pass)."""
    gen = torch.Generator().manual_seed(sum(shape) + 7 * res + relu)
    y = torch.randn(shape, generator=gen).cuda() * 4
    y.view(-1)[:3] = torch.tensor([-0.0, float("nan"), 0.0])
    y.view(-1)[3:6] = torch.tensor([6.0, 6.0000005, 5.9999995])
    b = torch.randn(shape[1], generator=gen).cuda()
    b[0] = 0.0
    r = torch.randn(shape, generator=gen).cuda() if res else None
    if res:
        r.view(-1)[:6] = 0.0
    d = torch.tensor(0.21).cuda()
    z = torch.tensor(3.0).cuda()
    g = torch.randn(shape, generator=gen).cuda()
    with torch.no_grad():
        a = K.bias_act_quant(y, b, r, relu, d, z, 4)
    results = []
    for fused in (True, False):
        yy = y.clone().requires_grad_(True)
        rr = r.clone().requires_grad_(True) if res else None
        dd = d.clone().requires_grad_(True)
        zz = z.clone().requires_grad_(True)
        if fused:
            o = K.bias_act_quant(yy, b, rr, relu, dd, zz, 4)
        else:
            o = K.fake_quant(K.bias_act(yy, b, rr, relu), dd, zz, 4)
        o.backward(g)
        results.append([host(o), host(yy.grad), host(dd.grad), host(zz.grad)]
                       + ([host(rr.grad)] if res else []))
    np.testing.assert_array_equal(host(a).view(np.int32), results[0][0].view(np.int32))
    for u, v in zip(*results):
        np.testing.assert_array_equal(np.asarray(u).view(np.int32), np.asarray(v).view(np.int32))


def test_lp_loss_relu_mask_folds_relu_backward(K):
    """lp_loss(relu(t), tgt) with relu_mask: the gradient written is d loss / d t, equal
    to torch autograd through the ReLU of the unmasked lp gradient, bit for bit."""
    gen = torch.Generator().manual_seed(21)
    t = torch.randn(8, 16, 9, 9, generator=gen).cuda()
    t.view(-1)[:2] = torch.tensor([0.0, -0.0])
    out = torch.relu(t)
    tgt = torch.randn(8, 16, 9, 9, generator=gen).cuda()
    l1, g_plain = K.lp_loss_and_grad(out, tgt, 2.0)
    l2, g_mask = K.lp_loss_and_grad(out, tgt, 2.0, relu_mask=True)
    assert host(l1) == host(l2)
    ref = torch.where(out <= 0, torch.zeros_like(g_plain), g_plain)
    np.testing.assert_array_equal(host(g_mask), host(ref))


def test_ssq_adam_matches_torch_single_tensor_adam(K):
    """SsqAdam (one ssq_adam launch) follows torch.optim.Adam's single-tensor update (the
    reference's optimizer on CPU) over 50 steps, with host and device hyper-parameters."""
    from shiftedscalequantization_amd.quant._engine import SsqAdam
    gen = torch.Generator().manual_seed(4)
    shapes = [(64, 3), (5,), (7, 9, 3)]
    ref = [torch.randn(s, generator=gen).requires_grad_(True) for s in shapes]
    mine = [p.detach().clone().cuda().requires_grad_(True) for p in ref]
    mine2 = [p.detach().clone().cuda().requires_grad_(True) for p in ref]
    topt = torch.optim.Adam(ref, lr=3e-3, foreach=False)
    sopt, sopt2 = SsqAdam(mine, lr=3e-3), SsqAdam(mine2, lr=3e-3)
    hyper = torch.zeros(2, device="cuda")
    for it in range(50):
        grads = [torch.randn(s, generator=gen) * (0.1 if it % 7 else 1e-6) for s in shapes]
        for p, g in zip(ref, grads):
            p.grad = g.clone()
        for p, g in zip(mine, grads):
            p.grad = g.cuda()
        for p, g in zip(mine2, grads):
            p.grad = g.cuda()
        topt.step()
        sopt.step()
        hyper.copy_(torch.tensor(sopt2.next_hyper(), dtype=torch.float32))
        sopt2.step(hyper=hyper)
    for a, b, c in zip(ref, mine, mine2):
        np.testing.assert_allclose(host(b), a.detach().numpy(), rtol=2e-6, atol=1e-7)
        np.testing.assert_array_equal(host(b), host(c))


@pytest.mark.parametrize("n", [4096 * 33, 4099, 12])
def test_fq_bwd_per_tensor_vs_oracle(K, n):
    """Per-tensor STE backward (float4 and scalar forms): gx bit-exact, delta / zero_point
    gradients within 1e-5 of the oracle's double sums."""
    gen = torch.Generator().manual_seed(n)
    x = torch.relu(torch.randn(n, generator=gen)) * 3
    gy = torch.randn(n, generator=gen)
    d, z = torch.tensor(0.21), torch.tensor(1.0)
    xr = x.cuda().requires_grad_(True)
    dd = d.cuda().requires_grad_(True)
    zz = z.cuda().requires_grad_(True)
    y = K.fake_quant(xr, dd, zz, 4, False)
    y.backward(gy.cuda())
    rgx, rgd, rgz = R.fake_quant_bwd(x.numpy(), d.numpy(), z.numpy(), 4, False, gy.numpy())
    np.testing.assert_array_equal(host(xr.grad), rgx)
    close(host(dd.grad).reshape(-1), np.reshape(rgd, -1), rtol=1e-5, atol=1e-6)
    close(host(zz.grad).reshape(-1), np.reshape(rgz, -1), rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("d", [0.21, 2.0 ** -40, 3.0e9])
def test_fq_bwd_extreme_values_bit_exact(K, d):
    """fq_bwd_pt4 (the float4 STE backward) with values planted far outside the usual range
    (tiny, huge, zeros, inf, NaN) and deltas from 2^-40 to 3e9: gx bit-exact against numpy's
    IEEE fp32, the delta / zero-point gradients (the (x/d)/d term with two IEEE divides) as
    the oracle's float64 sums."""
    n = 1 << 20
    gen = torch.Generator().manual_seed(int(d * 1e3) % 1000 + 7)
    x = (torch.randn(n, generator=gen) * 4 * d).float()
    gy = torch.randn(n, generator=gen)
    pos = torch.randperm(n, generator=gen)[:24]
    specials = torch.tensor([1e-38, -3e-39, 2.0 ** -31, 2.0 ** 31, 1e30, -1e33, 0.0, -0.0,
                             float("inf"), float("-inf"), float("nan"), 1e-20])
    x[pos[:12]] = specials * (d if d < 1 else 1.0)
    gy[pos[12:]] = specials
    d_t, z_t = torch.tensor(np.float32(d)), torch.tensor(3.0)
    xr = x.cuda().requires_grad_(True)
    dd, zz = d_t.cuda().requires_grad_(True), z_t.cuda().requires_grad_(True)
    K.fake_quant(xr, dd, zz, 4, False).backward(gy.cuda())
    rgx, rgd, rgz = R.fake_quant_bwd(x.numpy(), d_t.numpy(), z_t.numpy(), 4, False, gy.numpy())
    np.testing.assert_array_equal(host(xr.grad).view(np.int32), np.asarray(rgx, np.float32).view(np.int32))
    for got, ref in ((host(dd.grad), rgd), (host(zz.grad), rgz)):
        got, ref = np.reshape(got, -1), np.reshape(ref, -1)
        assert np.array_equal(np.isnan(got), np.isnan(ref))
        ok = ~np.isnan(ref)
        close(got[ok], ref[ok], rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("level,threshold", [(1024, 2.0), (64, 1.0), (1, 1.5), (333, 0.5)])
def test_inpscale_search_binary_search_equals_scan(K, level, threshold):
    """The kernel's binary search over k returns exactly the reference's linear scan
    (the oracle) -- every column, including ones where no candidate fits."""
    gen = torch.Generator().manual_seed(level)
    w = torch.randn(96, 32, 3, 3, generator=gen) * 0.05
    w[:, 0] *= 40.0                                # columns where only c = 1 (or none) fits
    d, z, raw = R.init_scale(w.numpy(), 2, False, True, "max")
    inp = K.inpscale_search(w.cuda(), dev(d).view(-1, 1, 1, 1), dev(raw).view(-1, 1, 1, 1), 2, level,
                            threshold)
    ref = R.inpscale_search(w.numpy(), d.reshape(-1, 1, 1, 1), raw.reshape(-1, 1, 1, 1), 2, level,
                            threshold)
    np.testing.assert_array_equal(host(inp), ref)


@pytest.mark.parametrize("row_shape", [(16, 7, 7), (3, 5, 3), (64, 14, 14)])
@pytest.mark.parametrize("p", [2.0, 2.4, 1.0])
def test_lp_loss_rows_equals_gathered(K, row_shape, p):
    """Loss pass reading cache[idx] in place (ssq_lp_loss_rows) == gather + ssq_lp_loss,
    bit for bit (value and gradient, with and without the ReLU mask)."""
    gen = torch.Generator().manual_seed(len(row_shape) + int(p * 10))
    cache = torch.randn((40,) + row_shape, generator=gen).cuda()
    idx = torch.randperm(40, generator=gen)[:8].cuda()
    pred = torch.relu(torch.randn((8,) + row_shape, generator=gen)).cuda()
    tgt = K.gather_rows2(cache, idx)[0]
    for relu_mask in (False, True):
        l1, g1 = K.lp_loss_and_grad(pred, tgt, p, relu_mask=relu_mask)
        l2, g2 = K.lp_loss_and_grad(pred, K.Rows(cache, idx), p, relu_mask=relu_mask)
        assert host(l1).tobytes() == host(l2).tobytes()
        np.testing.assert_array_equal(host(g1).view(np.int32), host(g2).view(np.int32))


@pytest.fixture(params=[1, 2, 3, 4], ids=["tile", "i2c", "band", "band4w"])
def wgrad_form(request):
    from shiftedscalequantization_amd import kernels
    old = kernels.set_wgrad_form(request.param)
    yield request.param
    kernels.set_wgrad_form(old)


@pytest.mark.parametrize("cfg", [
    # (Nb, C, H, Co, k, stride, pad, groups)
    (4, 64, 56, 64, 3, 1, 1, 1), (3, 16, 15, 24, 3, 2, 1, 1), (2, 32, 14, 48, 1, 2, 0, 1),
    (2, 24, 9, 24, 3, 1, 1, 24), (2, 48, 12, 96, 3, 1, 1, 2), (5, 130, 7, 70, 3, 1, 1, 1),
    (1, 3, 32, 16, 7, 2, 3, 1),
    # GEMM path layouts: few input channels (WM = 4 tiles), rows wider than a wave and than
    # a chunk, 7x7 planes (short chunks), stride 2 at 28x28
    (2, 16, 14, 256, 1, 1, 0, 1), (1, 8, 70, 16, 3, 1, 1, 1), (1, 4, 130, 8, 3, 1, 1, 1),
    (2, 256, 7, 512, 3, 1, 1, 1), (2, 64, 28, 128, 3, 2, 1, 1),
    # band path (3x3 pad 1, OW % 4 == 0): ResNet layer1 / layer2 / layer2.0 stride 2,
    # ragged output-channel tiles, fewer input channels than the tile, one-row bands
    (3, 128, 28, 128, 3, 1, 1, 1), (2, 64, 56, 128, 3, 2, 1, 1), (2, 32, 16, 96, 3, 2, 1, 1),
    (3, 32, 8, 160, 3, 1, 1, 1), (2, 96, 12, 64, 3, 1, 1, 1),
    # band path on small planes: 2 / 1 pixels per step, 4-byte DMA (rows not 16-B aligned),
    # bands padded to the two lane halves: ResNet layer3 / layer3.0 s2 / layer4 / layer4.0 s2,
    # odd planes
    (2, 256, 14, 256, 3, 1, 1, 1), (2, 128, 28, 256, 3, 2, 1, 1), (3, 512, 7, 512, 3, 1, 1, 1),
    (2, 256, 14, 512, 3, 2, 1, 1), (2, 32, 9, 64, 3, 1, 1, 1), (2, 64, 10, 96, 3, 2, 1, 1),
    (1, 32, 6, 32, 3, 1, 1, 1),
    # 1x1 GEMM path: ResNet downsamples (stride 2 at 56x56 / 14x14), ragged channel
    # counts over the 128 x 128 tile, grouped, a plane shorter than one chunk
    (2, 64, 56, 128, 1, 2, 0, 1), (2, 256, 14, 512, 1, 2, 0, 1), (3, 72, 9, 40, 1, 1, 0, 1),
    (2, 300, 7, 130, 1, 1, 0, 1), (2, 48, 12, 96, 1, 1, 0, 2), (4, 16, 5, 24, 1, 2, 0, 1),
    # depthwise path: stride 2, planes wider than a wave, 5x5, odd batch
    (3, 32, 57, 32, 3, 2, 1, 32), (2, 144, 28, 144, 3, 1, 1, 144), (5, 16, 11, 16, 5, 1, 2, 16),
    (32, 8, 7, 8, 3, 1, 1, 8),
    # depthwise, several samples staged per pass: MobileNetV2 features.16 (16 samples of a
    # 7x7 plane in one pass), a ragged last pass (11 samples, 9 per pass), 5x5 on 14x14
    (32, 960, 7, 960, 3, 1, 1, 960), (11, 520, 28, 520, 3, 2, 1, 520),
    (8, 400, 14, 400, 5, 1, 2, 400),
    # depthwise on planes cut into row bands: 112x112 (8 bands, a short last one), 5x5
    # stride 2 (3 bands)
    (2, 16, 112, 16, 3, 1, 1, 16), (2, 8, 64, 8, 5, 2, 2, 8)])
def test_conv_wgrad_matches_fp64(K, cfg, wgrad_form):
    """K17 weight gradient (both non-depthwise forms) vs the fp64 CPU gradient: error
    within the fp32 accumulation bound, bit-identical run to run, and the autograd wrapper
    equals the direct call."""
    Nb, C, H, Co, k, st, pad, g = cfg
    gen = torch.Generator().manual_seed(sum(cfg))
    x = torch.randn(Nb, C, H, H, generator=gen)
    w = torch.randn(Co, C // g, k, k, generator=gen)
    y = torch.nn.functional.conv2d(x, w, None, st, pad, 1, g)
    dy = torch.randn(y.shape, generator=gen)
    ref = torch.nn.grad.conv2d_weight(x.double(), w.shape, dy.double(), st, pad, 1, g)
    mag = torch.nn.grad.conv2d_weight(x.double().abs(), w.shape, dy.double().abs(), st, pad, 1, g)
    xd, dyd = x.cuda(), dy.cuda()
    dw1 = K.conv_wgrad(xd, dyd, w.shape, st, pad, g)
    dw2 = K.conv_wgrad(xd, dyd, w.shape, st, pad, g)
    np.testing.assert_array_equal(host(dw1).view(np.int32), host(dw2).view(np.int32))
    err = (dw1.double().cpu() - ref).abs()
    assert bool((err <= 1e-5 * mag + 1e-30).all()), float((err / mag.clamp_min(1e-30)).max())
    wd = w.cuda().requires_grad_(True)
    old, K.WGRAD_POLICY = K.WGRAD_POLICY, "always"
    old_gemm, K.WGRAD_GEMM = K.WGRAD_GEMM, "never"
    try:
        out = K.conv2d(xd, wd, st, pad, 1, g)
        out.backward(dyd)
    finally:
        K.WGRAD_POLICY, K.WGRAD_GEMM = old, old_gemm
    np.testing.assert_array_equal(host(wd.grad).view(np.int32), host(dw1).view(np.int32))


@pytest.mark.parametrize("cfg", [
    # (Nb, C, H, Co, stride): ResNet-18 layer1 / layer2.0 s2 / layer2 / layer3.0 s2 (16-B
    # staging), layer3 / layer4 (4-B staging, 2 / 1 pixels per step), ragged tiles
    (32, 64, 56, 64, 1), (8, 64, 56, 128, 2), (8, 128, 28, 128, 1), (8, 128, 28, 256, 2),
    (4, 256, 14, 256, 1), (4, 512, 7, 512, 1), (3, 32, 8, 160, 1), (2, 96, 12, 64, 1)])
def test_band_wgrad_two_waves_per_simd_bit_identical(K, cfg):
    """The band kernel at 8 waves per workgroup (two per SIMD, the taps split 5 / 4 between
    the waves of a tile) gives the 4-wave kernel's bits: every tap sums the same pixels in
    the same order."""
    Nb, C, H, Co, st = cfg
    gen = torch.Generator().manual_seed(sum(cfg))
    x = torch.randn(Nb, C, H, H, generator=gen).cuda()
    oh = (H - 1) // st + 1
    dy = torch.randn(Nb, Co, oh, oh, generator=gen).cuda()
    old = K.set_wgrad_form(3)
    try:
        assert K.wgrad_kind(x.shape, (Co, C, 3, 3), st, 1, 1) in (3, 6)
        dw8 = K.conv_wgrad(x, dy, (Co, C, 3, 3), st, 1, 1)
        K.set_wgrad_form(4)
        dw4 = K.conv_wgrad(x, dy, (Co, C, 3, 3), st, 1, 1)
    finally:
        K.set_wgrad_form(old)
    np.testing.assert_array_equal(host(dw8).view(np.int32), host(dw4).view(np.int32))


@pytest.mark.parametrize("cfg", [
    # (N, C, H, W, k, stride, pad): the ResNet stem's pool at batch 8, odd planes, 2x2 / s2,
    # 3x3 / s1, 5x5 / s2 / p2, a 7x7 window over a 7x7 plane
    (8, 64, 112, 112, 3, 2, 1), (3, 5, 17, 13, 3, 2, 1), (2, 4, 8, 8, 2, 2, 0),
    (2, 3, 9, 11, 3, 1, 1), (1, 6, 15, 15, 5, 2, 2), (2, 2, 7, 7, 7, 1, 3),
    # the two-outputs-per-thread 3x3 / s2 / p1 form (even W and OW): small and odd H
    (2, 3, 6, 8, 3, 2, 1), (3, 2, 5, 4, 3, 2, 1)])
def test_maxpool2d_matches_torch(K, cfg):
    """ssq_maxpool2d_fwd (SsqMaxPool2d, the stem's pool in QuantModel) == torch's
    F.max_pool2d bit for bit, NaN / inf / signed zeros / ties included; the module takes
    torch's path where a gradient is needed."""
    N, C, H, W, k, st, pad = cfg
    gen = torch.Generator().manual_seed(sum(cfg))
    x = torch.randn(N, C, H, W, generator=gen)
    x.view(-1)[:8] = torch.tensor([float("nan"), -0.0, 0.0, float("inf"), -float("inf"),
                                   1.0, 1.0, -0.0])
    x[0, 0, 1, :] = 0.0
    x[0, 0, 2, ::2] = -0.0
    xd = x.cuda()
    ref = torch.nn.functional.max_pool2d(xd, k, st, pad)
    y = K.maxpool2d(xd, k, st, pad)
    np.testing.assert_array_equal(host(y).view(np.int32), host(ref).view(np.int32))
    m = K.SsqMaxPool2d.wrap(torch.nn.MaxPool2d(k, st, pad))
    with torch.no_grad():
        np.testing.assert_array_equal(host(m(xd)).view(np.int32), host(ref).view(np.int32))
    xg = xd.clone().requires_grad_(True)
    out = m(xg)
    assert out.grad_fn is not None
    out.sum().backward()
    assert xg.grad is not None


@pytest.mark.parametrize("cfg", [
    # (Nb, C, H, Co): ResNet-18 downsamples at batch 32 (layer2.0 / layer4.0: batched GEMM;
    # layer3.0: MIOpen below batch 128), layer3.0 at batch 128, odd sizes
    (32, 64, 56, 128), (32, 256, 14, 512), (32, 128, 28, 256), (128, 128, 28, 256),
    (3, 40, 9, 24)])
def test_conv1x1_stride2_forward_gemm(K, cfg):
    """1x1 stride-2 forward as one strided-batched GEMM (FWD_1X1_GEMM) vs the fp64 conv within
    the fp32 accumulation bound, bit-identical run to run, taken by K.conv2d with and without
    grad exactly where the policy says, and the autograd path's gradients unchanged (MIOpen
    input gradient, K17 / GEMM weight gradient)."""
    Nb, C, H, Co = cfg
    gen = torch.Generator().manual_seed(sum(cfg))
    x = torch.randn(Nb, C, H, H, generator=gen)
    w = torch.randn(Co, C, 1, 1, generator=gen) * 0.05
    ref = torch.nn.functional.conv2d(x.double(), w.double(), None, 2)
    mag = torch.nn.functional.conv2d(x.double().abs(), w.double().abs(), None, 2)
    xd, wd = x.cuda(), w.cuda()
    use = K._use_fwd_1x1(xd, wd, 2, 0, 1, 1)
    assert use == (not (100 < ((H + 1) // 2) ** 2 < 400 and Nb < 128))
    y1, y2 = K.conv1x1_fwd_gemm(xd, wd, 2), K.conv1x1_fwd_gemm(xd, wd, 2)
    np.testing.assert_array_equal(host(y1).view(np.int32), host(y2).view(np.int32))
    err = (y1.double().cpu() - ref).abs()
    assert bool((err <= 1e-5 * mag + 1e-30).all())
    with torch.no_grad():
        y3 = K.conv2d(xd, wd, 2, 0)
    if use:
        np.testing.assert_array_equal(host(y3).view(np.int32), host(y1).view(np.int32))
    assert bool(((y3.double().cpu() - ref).abs() <= 1e-5 * mag + 1e-30).all())
    # training path under the reference's cudnn.deterministic (Conv2dFn): same forward, and
    # the gradients of the MIOpen-forward path
    old_det = torch.backends.cudnn.deterministic
    old, K.FWD_1X1_GEMM = K.FWD_1X1_GEMM, True
    torch.backends.cudnn.deterministic = True
    try:
        xg = xd.clone().requires_grad_(True)
        wg = wd.clone().requires_grad_(True)
        yg = K.conv2d(xg, wg, 2, 0)
        if use:
            np.testing.assert_array_equal(host(yg.detach()).view(np.int32), host(y1).view(np.int32))
        dy = torch.randn(yg.shape, generator=gen).cuda()
        yg.backward(dy)
        K.FWD_1X1_GEMM = False
        xm = xd.clone().requires_grad_(True)
        wm = wd.clone().requires_grad_(True)
        K.conv2d(xm, wm, 2, 0).backward(dy)
    finally:
        K.FWD_1X1_GEMM = old
        torch.backends.cudnn.deterministic = old_det
    np.testing.assert_array_equal(host(xg.grad).view(np.int32), host(xm.grad).view(np.int32))
    if use and K._use_wgrad_bmm_s2(xd, wd, 2, 0):
        # the weight gradient then runs on the forward's subsampled input (WGRAD_S2_BMM,
        # test_conv_wgrad_s2_bmm_matches_fp64): another summation order, same bound
        rw = torch.nn.grad.conv2d_weight(x.double(), w.shape, dy.double().cpu(), 2, 0)
        mw = torch.nn.grad.conv2d_weight(x.double().abs(), w.shape, dy.double().abs().cpu(), 2, 0)
        for gw in (wg.grad, wm.grad):
            assert bool(((gw.double().cpu() - rw).abs() <= 1e-5 * mw + 1e-30).all())
    else:
        np.testing.assert_array_equal(host(wg.grad).view(np.int32), host(wm.grad).view(np.int32))


@pytest.mark.parametrize("cfg", [
    # (Nb, C, H, Co): ResNet-50 layer1.0's conv1 / conv3+downsample, RegNetX-3200M s3.b1 'a',
    # MobileNetV2's 56x56 expand, ragged sizes at the 400-pixel edge
    (32, 64, 56, 64), (32, 64, 56, 256), (32, 192, 28, 432), (32, 24, 56, 144), (3, 37, 20, 29),
    (4, 16, 19, 8)])
def test_conv_wgrad_1x1_bmm_matches_fp64(K, cfg):
    """The 1x1 stride-1 weight gradient on planes >= 400 pixels as one strided-batched GEMM
    and an in-order batch sum (K.conv_wgrad_1x1_bmm, WGRAD_1X1_BMM): vs the fp64 CPU gradient
    within the fp32 accumulation bound, bit-identical run to run, and what K.conv2d's
    training path (Conv2dFn under cudnn.deterministic) hands the weight -- below 400 pixels,
    or with the policy forced, K17 / the im2col GEMM as before."""
    Nb, C, H, Co = cfg
    gen = torch.Generator().manual_seed(sum(cfg))
    x = torch.relu(torch.randn(Nb, C, H, H, generator=gen))
    w = torch.randn(Co, C, 1, 1, generator=gen) * 0.1
    dy = torch.randn(Nb, Co, H, H, generator=gen)
    ref = torch.nn.grad.conv2d_weight(x.double(), w.shape, dy.double(), 1, 0)
    mag = torch.nn.grad.conv2d_weight(x.double().abs(), w.shape, dy.double().abs(), 1, 0)
    xd, dyd = x.cuda(), dy.cuda()
    dw1, dw2 = K.conv_wgrad_1x1_bmm(xd, dyd, w.shape), K.conv_wgrad_1x1_bmm(xd, dyd, w.shape)
    np.testing.assert_array_equal(host(dw1).view(np.int32), host(dw2).view(np.int32))
    err = (dw1.double().cpu() - ref).abs()
    assert bool((err <= 1e-5 * mag + 1e-30).all()), float((err / mag.clamp_min(1e-30)).max())
    wd = w.cuda()
    old_det = torch.backends.cudnn.deterministic
    try:
        torch.backends.cudnn.deterministic = False
        assert K._use_wgrad_bmm(xd, wd, 1, 0) == (H * H >= 400)
        torch.backends.cudnn.deterministic = True  # 14x14 planes and up there
        assert K._use_wgrad_bmm(xd, wd, 1, 0) == (H * H >= 100)
        wg = wd.clone().requires_grad_(True)
        K.conv2d(xd, wg, 1, 0).backward(dyd)
    finally:
        torch.backends.cudnn.deterministic = old_det
    if H * H >= 100:
        np.testing.assert_array_equal(host(wg.grad).view(np.int32), host(dw1).view(np.int32))
    assert bool(((wg.grad.double().cpu() - ref).abs() <= 1e-5 * mag + 1e-30).all())


@pytest.mark.parametrize("cfg", [
    # (Nb, C, H, Co, bmm?): ResNet-18 layer2.0's downsample (28x28 out), a 64-multiple one at
    # the 400-pixel edge, RegNetX s2.b1's 96 -> 192 (K17 keeps it), a 14x14 one (im2col GEMM)
    (32, 64, 56, 128, True), (3, 64, 40, 64, True), (4, 96, 56, 192, False),
    (4, 128, 28, 256, False)])
def test_conv_wgrad_s2_bmm_matches_fp64(K, cfg):
    """1x1 stride-2 weight gradients as one batched GEMM + batch sum over the subsampled
    input the forward GEMM made contiguous (WGRAD_S2_BMM): K.conv2d's training path under
    cudnn.deterministic hands the weight exactly K.conv_wgrad_1x1_bmm(xs)'s bits where the
    rule takes the shape, and every route is within the fp32 bound of the fp64 gradient."""
    Nb, C, H, Co, bmm = cfg
    gen = torch.Generator().manual_seed(Nb + C + H + Co)
    x = torch.relu(torch.randn(Nb, C, H, H, generator=gen))
    w = torch.randn(Co, C, 1, 1, generator=gen) * 0.1
    dy = torch.randn(Nb, Co, H // 2, H // 2, generator=gen)
    ref = torch.nn.grad.conv2d_weight(x.double(), w.shape, dy.double(), 2, 0)
    mag = torch.nn.grad.conv2d_weight(x.double().abs(), w.shape, dy.double().abs(), 2, 0)
    xd, wd, dyd = x.cuda(), w.cuda(), dy.cuda()
    assert K._use_wgrad_bmm_s2(xd, wd, 2, 0) == bmm
    old_det = torch.backends.cudnn.deterministic
    torch.backends.cudnn.deterministic = True
    try:
        wg = wd.clone().requires_grad_(True)
        y = K.conv2d(xd, wg, 2, 0)
        y.backward(dyd)
    finally:
        torch.backends.cudnn.deterministic = old_det
    if bmm:
        xs = xd[:, :, ::2, ::2].contiguous()
        gw = K.conv_wgrad_1x1_bmm(xs, dyd, w.shape)
        np.testing.assert_array_equal(host(wg.grad).view(np.int32), host(gw).view(np.int32))
    assert bool(((wg.grad.double().cpu() - ref).abs() <= 1e-5 * mag + 1e-30).all())
    yref = torch.nn.functional.conv2d(x.double(), w.double(), None, 2)
    ymag = torch.nn.functional.conv2d(x.double().abs(), w.double().abs(), None, 2)
    assert bool(((y.detach().double().cpu() - yref).abs() <= 1e-5 * ymag + 1e-30).all())


def test_gemm_operands_noncontiguous_inputs(K):
    """ssq_wgrad_gemm_operands from non-contiguous x and dy (channels-last x, a transposed
    view of dy): both are copied to contiguous tensors held until the launch -- the operands
    equal those of the contiguous inputs, bit for bit."""
    gen = torch.Generator().manual_seed(11)
    x = torch.randn(4, 16, 9, 9, generator=gen).cuda()
    dy = torch.randn(4, 24, 9, 9, generator=gen).cuda()
    xn = x.to(memory_format=torch.channels_last)
    dyn = dy.transpose(2, 3).contiguous().transpose(2, 3)
    assert not xn.is_contiguous() and not dyn.is_contiguous()
    c1, d1 = K.gemm_operands(x, dy, (24, 16, 3, 3), 1, 1)
    c2, d2 = K.gemm_operands(xn, dyn, (24, 16, 3, 3), 1, 1)
    np.testing.assert_array_equal(host(c1).view(np.int32), host(c2).view(np.int32))
    np.testing.assert_array_equal(host(d1).view(np.int32), host(d2).view(np.int32))


@pytest.mark.parametrize("cfg", [
    # (Nb, C, H, Co, GEMM?): MobileNetV2 features.16's project (960 -> 160 on 7x7: GEMM) and
    # expand (MIOpen), features.2's 112x112 expand, ResNet-50 layer3's expand (14x14),
    # layer1.0 conv3 (56x56: MIOpen), a ragged one
    (32, 960, 7, 160, True), (32, 160, 7, 960, False), (32, 16, 112, 96, True),
    (32, 256, 14, 1024, True), (32, 64, 56, 256, False), (3, 37, 9, 29, False)])
@pytest.mark.parametrize("weight_grad", [True, False], ids=["weight_phase", "act_phase"])
def test_conv1x1_dgrad_gemm_matches_fp64(K, cfg, weight_grad):
    """The input gradient of 1x1 stride-1 convs as one strided-batched GEMM
    (K.conv1x1_dgrad_gemm, DGRAD_1X1_GEMM, on the shapes its rule names): vs the fp64 CPU
    gradient within the fp32 accumulation bound, bit-identical run to run, and what K.conv2d's
    autograd hands the input under cudnn.deterministic, with the weight trained (Conv2dFn) and
    fixed (an activation-phase conv): the GEMM's bits where the rule takes the shape, else
    MIOpen's within the same bound; and the weight's gradient within it too."""
    Nb, C, H, Co, gemm = cfg
    gen = torch.Generator().manual_seed(Nb + C + H + Co + 7)
    x = torch.relu(torch.randn(Nb, C, H, H, generator=gen))
    w = torch.randn(Co, C, 1, 1, generator=gen) * 0.1
    dy = torch.randn(Nb, Co, H, H, generator=gen)
    ref = torch.nn.grad.conv2d_input(x.shape, w.double(), dy.double(), 1, 0)
    mag = torch.nn.grad.conv2d_input(x.shape, w.double().abs(), dy.double().abs(), 1, 0)
    xd, wd, dyd = x.cuda(), w.cuda(), dy.cuda()
    g1, g2 = K.conv1x1_dgrad_gemm(dyd, wd), K.conv1x1_dgrad_gemm(dyd, wd)
    np.testing.assert_array_equal(host(g1).view(np.int32), host(g2).view(np.int32))
    assert bool(((g1.double().cpu() - ref).abs() <= 1e-5 * mag + 1e-30).all())
    old_det = torch.backends.cudnn.deterministic
    try:
        torch.backends.cudnn.deterministic = False
        assert not K._use_dgrad_1x1(xd, wd, 1, 0)
        torch.backends.cudnn.deterministic = True
        assert K._use_dgrad_1x1(xd, wd, 1, 0) == gemm
        xg = xd.clone().requires_grad_(True)
        wg = wd.clone().requires_grad_(weight_grad)
        K.conv2d(xg, wg, 1, 0).backward(dyd)
    finally:
        torch.backends.cudnn.deterministic = old_det
    if gemm:
        np.testing.assert_array_equal(host(xg.grad).view(np.int32), host(g1).view(np.int32))
    assert bool(((xg.grad.double().cpu() - ref).abs() <= 1e-5 * mag + 1e-30).all())
    if weight_grad:
        rw = torch.nn.grad.conv2d_weight(x.double(), w.shape, dy.double(), 1, 0)
        mw = torch.nn.grad.conv2d_weight(x.double().abs(), w.shape, dy.double().abs(), 1, 0)
        assert bool(((wg.grad.double().cpu() - rw).abs() <= 1e-5 * mw + 1e-30).all())


@pytest.mark.parametrize("cfg", [
    # (Nb, C, H, stride, groups): RegNetX-3200M s3.b1 / s3.b2 / s4.b2 'b' convs (group width
    # 48), a ragged one, and s2.b2's 28x28 plane (K17 keeps it)
    (32, 432, 28, 2, 9), (32, 432, 14, 1, 9), (32, 1008, 7, 1, 21), (3, 36, 9, 1, 3),
    (8, 192, 28, 1, 4)])
def test_conv_wgrad_grouped_gemm_matches_fp64(K, cfg):
    """Grouped-conv weight gradients on output planes <= 196 pixels as the im2col operands of
    every channel and one strided-batched GEMM over the groups (K.conv_wgrad_grouped_gemm,
    WGRAD_GROUPED_GEMM): vs the fp64 CPU gradient within the fp32 accumulation bound,
    bit-identical run to run, and what K.conv2d's training path hands the weight (larger
    planes: K17 as before); the forward as one GEMM over the groups on the same im2col
    matrix (K.conv_fwd_grouped_gemm) likewise, and the weight gradient from its saved
    matrix bit-identical to the one built in the backward."""
    Nb, C, H, st, G = cfg
    gen = torch.Generator().manual_seed(sum(cfg))
    w_shape = (C, C // G, 3, 3)
    x = torch.relu(torch.randn(Nb, C, H, H, generator=gen))
    w = torch.randn(w_shape, generator=gen) * 0.1
    y = torch.nn.functional.conv2d(x, w, None, st, 1, 1, G)
    dy = torch.randn(y.shape, generator=gen)
    ref = torch.nn.grad.conv2d_weight(x.double(), w_shape, dy.double(), st, 1, groups=G)
    mag = torch.nn.grad.conv2d_weight(x.double().abs(), w_shape, dy.double().abs(), st, 1, groups=G)
    xd, dyd, wd = x.cuda(), dy.cuda(), w.cuda()
    small = y.shape[2] * y.shape[3] <= 196
    assert K._use_wgrad_grouped_gemm(xd, wd, st, 1, G) == small
    dw1 = K.conv_wgrad_grouped_gemm(xd, dyd, w_shape, st, 1, G)
    dw2 = K.conv_wgrad_grouped_gemm(xd, dyd, w_shape, st, 1, G)
    np.testing.assert_array_equal(host(dw1).view(np.int32), host(dw2).view(np.int32))
    err = (dw1.double().cpu() - ref).abs()
    assert bool((err <= 1e-5 * mag + 1e-30).all()), float((err / mag.clamp_min(1e-30)).max())
    # the forward as one GEMM over the groups on the same im2col matrix (GROUPED_GEMM_FWD)
    yref = torch.nn.functional.conv2d(x.double(), w.double(), None, st, 1, 1, G)
    ymag = torch.nn.functional.conv2d(x.double().abs(), w.double().abs(), None, st, 1, 1, G)
    if small:
        y1, col = K.conv_fwd_grouped_gemm(xd, wd, st, 1, G)
        y2, _ = K.conv_fwd_grouped_gemm(xd, wd, st, 1, G)
        np.testing.assert_array_equal(host(y1).view(np.int32), host(y2).view(np.int32))
        assert y1.shape == yref.shape and y1.is_contiguous()
        assert bool(((y1.double().cpu() - yref).abs() <= 1e-5 * ymag + 1e-30).all())
        dw3 = K.conv_wgrad_grouped_gemm(xd, dyd, w_shape, st, 1, G, col=col)
        np.testing.assert_array_equal(host(dw3).view(np.int32), host(dw1).view(np.int32))
    old_det = torch.backends.cudnn.deterministic
    torch.backends.cudnn.deterministic = True
    try:
        wg = wd.clone().requires_grad_(True)
        yo = K.conv2d(xd, wg, st, 1, 1, G)
        yo.backward(dyd)
    finally:
        torch.backends.cudnn.deterministic = old_det
    if small:
        np.testing.assert_array_equal(host(wg.grad).view(np.int32), host(dw1).view(np.int32))
        np.testing.assert_array_equal(host(yo.detach()).view(np.int32), host(y1).view(np.int32))
    assert bool(((wg.grad.double().cpu() - ref).abs() <= 1e-5 * mag + 1e-30).all())
    assert bool(((yo.detach().double().cpu() - yref).abs() <= 1e-5 * ymag + 1e-30).all())


@pytest.mark.parametrize("cfg", [
    # (Nb, C, H, Co, k, stride, pad): ResNet-18 layer3 / layer3.0 s2 / layer4 / layer4.0 s2
    # at batch 32 (the shapes the GEMM policy takes), a 5x5 and ragged sizes
    (32, 256, 14, 256, 3, 1, 1), (32, 128, 28, 256, 3, 2, 1), (32, 512, 7, 512, 3, 1, 1),
    (32, 256, 14, 512, 3, 2, 1), (3, 130, 9, 140, 3, 1, 1), (2, 64, 11, 128, 5, 2, 2),
    # 1x1 stride-2 downsamples of layer3.0 / layer4.0 (weight gradient only)
    (32, 128, 28, 256, 1, 2, 0), (32, 256, 14, 512, 1, 2, 0)])
def test_conv_wgrad_gemm_matches_fp64(K, cfg):
    """The im2col + library-GEMM weight gradient (ssq_wgrad_gemm_operands + hipBLASLt) vs
    the fp64 CPU gradient within the fp32 accumulation bound; its operands equal a host
    im2col / permute exactly; bit-identical run to run; K.conv2d routes the policy's
    shapes to it, with the forward as the GEMM over the same im2col matrix (vs the fp64
    conv) and the input gradient unchanged."""
    Nb, C, H, Co, k, st, pad = cfg
    gen = torch.Generator().manual_seed(sum(cfg))
    x = torch.randn(Nb, C, H, H, generator=gen)
    w = torch.randn(Co, C, k, k, generator=gen)
    y = torch.nn.functional.conv2d(x, w, None, st, pad)
    dy = torch.randn(y.shape, generator=gen)
    ref = torch.nn.grad.conv2d_weight(x.double(), w.shape, dy.double(), st, pad)
    mag = torch.nn.grad.conv2d_weight(x.double().abs(), w.shape, dy.double().abs(), st, pad)
    xd, dyd = x.cuda(), dy.cuda()
    # the operands themselves, exactly
    OH = y.shape[2]
    NP = Nb * OH * OH
    col = torch.empty(NP, C * k * k, device="cuda")
    dy2 = torch.empty(Co, NP, device="cuda")
    K.call("ssq_wgrad_gemm_operands", K.C.c_void_p(xd.data_ptr()), K.C.c_void_p(dyd.data_ptr()),
           Nb, C, H, H, Co, k, k, st, pad, K.C.c_void_p(col.data_ptr()),
           K.C.c_void_p(dy2.data_ptr()), K.stream_of(xd))
    cref = torch.nn.functional.unfold(x, k, padding=pad, stride=st)        # (N, C*k*k, P)
    np.testing.assert_array_equal(host(col), cref.permute(0, 2, 1).reshape(NP, -1).numpy())
    np.testing.assert_array_equal(host(dy2), dy.permute(1, 0, 2, 3).reshape(Co, -1).numpy())
    dw1 = K.conv_wgrad_gemm(xd, dyd, w.shape, st, pad)
    dw2 = K.conv_wgrad_gemm(xd, dyd, w.shape, st, pad)
    np.testing.assert_array_equal(host(dw1).view(np.int32), host(dw2).view(np.int32))
    err = (dw1.double().cpu() - ref).abs()
    assert bool((err <= 1e-5 * mag + 1e-30).all()), float((err / mag.clamp_min(1e-30)).max())
    wd = w.cuda().requires_grad_(True)
    assert K._use_wgrad_gemm(xd, wd, st, pad) and K._use_fwd_gemm(xd, wd, st, pad) == (k > 1)
    out = K.conv2d(xd, wd, st, pad)
    # the forward runs as the GEMM too (K.WGRAD_GEMM_FWD): vs the fp64 conv
    yref = torch.nn.functional.conv2d(x.double(), w.double(), None, st, pad)
    ymag = torch.nn.functional.conv2d(x.double().abs(), w.double().abs(), None, st, pad)
    assert out.shape == yref.shape and out.is_contiguous()
    yerr = (out.detach().double().cpu() - yref).abs()
    assert bool((yerr <= 1e-5 * ymag + 1e-30).all()), float((yerr / ymag.clamp_min(1e-30)).max())
    out.backward(dyd)
    np.testing.assert_array_equal(host(wd.grad).view(np.int32), host(dw1).view(np.int32))
    # input gradient (MIOpen, from the saved input) vs the fp64 one (MIOpen may pick another
    # solver than for the plain conv's joint backward, so not bit-compared with it)
    xg = xd.clone().requires_grad_(True)
    K.conv2d(xg, w.cuda().requires_grad_(True), st, pad).backward(dyd)
    gref = torch.nn.grad.conv2d_input(x.shape, w.double(), dy.double(), st, pad)
    gmag = torch.nn.grad.conv2d_input(x.shape, w.double().abs(), dy.double().abs(), st, pad)
    gerr = (xg.grad.double().cpu() - gref).abs()
    assert bool((gerr <= 1e-5 * gmag + 1e-30).all()), float((gerr / gmag.clamp_min(1e-30)).max())


@pytest.mark.parametrize("cfg", [
    # (Nb, C, H, k, stride, pad): MobileNetV2's 3x3 s1 / s2, odd sizes, 5x5, wide plane
    (4, 144, 56, 3, 1, 1), (3, 96, 57, 3, 2, 1), (2, 32, 112, 3, 1, 1), (5, 16, 11, 5, 1, 2),
    (2, 24, 9, 3, 2, 0), (32, 8, 7, 3, 1, 1)])
def test_dwconv_matches_fp64(K, cfg):
    """K18 depthwise forward and input gradient vs fp64 torch: within the fp32 rounding
    bound of an R*S-term sum, bit-identical run to run; K.conv2d's autograd routes the
    depthwise conv through K18 (forward, dx) and K17 (dw)."""
    Nb, C, H, k, st, pad = cfg
    gen = torch.Generator().manual_seed(sum(cfg))
    x = torch.randn(Nb, C, H, H, generator=gen)
    w = torch.randn(C, 1, k, k, generator=gen)
    y64 = torch.nn.functional.conv2d(x.double(), w.double(), None, st, pad, 1, C)
    ymag = torch.nn.functional.conv2d(x.double().abs(), w.double().abs(), None, st, pad, 1, C)
    dy = torch.randn(y64.shape, generator=gen)
    dx64 = torch.nn.grad.conv2d_input(x.shape, w.double(), dy.double(), st, pad, 1, C)
    dxmag = torch.nn.grad.conv2d_input(x.shape, w.double().abs(), dy.double().abs(), st, pad, 1, C)
    xd, wd, dyd = x.cuda(), w.cuda(), dy.cuda()
    y1 = K.dwconv_fwd(xd, wd, st, pad)
    y2 = K.dwconv_fwd(xd, wd, st, pad)
    np.testing.assert_array_equal(host(y1).view(np.int32), host(y2).view(np.int32))
    err = (y1.double().cpu() - y64).abs()
    assert bool((err <= 1e-6 * ymag + 1e-30).all()), float((err / ymag.clamp_min(1e-30)).max())
    dx1 = K.dwconv_bwd_data(dyd, wd, x.shape, st, pad)
    err = (dx1.double().cpu() - dx64).abs()
    assert bool((err <= 1e-6 * dxmag + 1e-30).all()), float((err / dxmag.clamp_min(1e-30)).max())
    xg = xd.clone().requires_grad_(True)
    wg = wd.clone().requires_grad_(True)
    out = K.conv2d(xg, wg, st, pad, 1, C)
    np.testing.assert_array_equal(host(out).view(np.int32), host(y1).view(np.int32))
    out.backward(dyd)
    np.testing.assert_array_equal(host(xg.grad).view(np.int32), host(dx1).view(np.int32))
    dw = K.conv_wgrad(xd, dyd, w.shape, st, pad, C)
    np.testing.assert_array_equal(host(wg.grad).view(np.int32), host(dw).view(np.int32))


def test_affine_stays_live_after_raw_device_updates(K):
    """gamma^z/phi^z updated by a raw device write (fused Adam, graph replay: no torch
    version bump) after being trainable must still be applied once frozen again."""
    from shiftedscalequantization_amd import quant as Q
    torch.manual_seed(8)
    qm = Q.QuantModule(torch.nn.Conv2d(4, 8, 3, padding=1), {"n_bits": 4, "channel_wise": True},
                       {"n_bits": 8}).cuda()
    qm.set_quant_state(True, False)
    x = torch.randn(2, 4, 6, 6).cuda()
    with torch.no_grad():
        y0 = qm(x)                                   # identity affine (cached check)
    qm.alpha_out.requires_grad_(True)
    qm(x)                                            # trainable once (bias_cal loop)
    new = torch.linspace(0.5, 1.5, 8).view_as(qm.alpha_out).cuda()
    K.stream_copy(new, qm.alpha_out.data)            # raw write, no version bump
    qm.alpha_out.requires_grad_(False)
    with torch.no_grad():
        y1 = qm(x)
        w = qm.weight_quantizer(qm.weight)
        ref = torch.nn.functional.conv2d(x, w, qm.bias, 1, 1) * new + qm.beta_out
    assert not torch.equal(y0, y1)
    np.testing.assert_array_equal(host(y1).view(np.int32), host(ref).view(np.int32))


# ------------------------------------------------------------------ round 2: a10 init_v
@pytest.mark.parametrize("tag", CQ_TAGS)
def test_init_v_golden(K, golden, tag):
    """a10 ChannelQuant.init_v (channelQuant.py:201-213): alpha from the DEQUANTIZED
    'none'-mode candidates at delta*s_i (ssq_shift_init mode 1) vs the reference's alpha,
    through the ChannelQuant class (which also sets mode 'learned_hard_sigmoid')."""
    from shiftedscalequantization_amd import quant as Q
    g = golden("channelquant")
    w, is_fc, d, z, bits = _cq(g, tag)
    alpha, _, _ = K.shift_init(dev(w), dev(d), SHIFTS, zp=dev(z), n_bits=bits, mode=1)
    if not is_fc and w.shape[1] == 1:
        alpha = alpha.view(1, -1)
    close(host(alpha), g[tag + "_lhs_alpha0"], rtol=1e-5, atol=1e-6)   # log/mean ulps
    uaq = Q.UniformAffineQuantizer(n_bits=bits, channel_wise=True, ch=w.shape).cuda()
    shape = (-1, 1) if is_fc else (-1, 1, 1, 1)
    uaq.delta = torch.nn.Parameter(dev(g[tag + "_delta"]).view(shape))
    uaq.zero_point = torch.nn.Parameter(dev(g[tag + "_zp"]).view(shape))
    uaq.inited = True
    cq = Q.ChannelQuant(1.0, uaq=uaq, weight_tensor=dev(w), shiftTarget=SHIFTS, name=tag)
    cq.init_v(dev(w))
    assert cq.opt_mode == "learned_hard_sigmoid"
    close(host(cq.alpha), g[tag + "_lhs_alpha0"], rtol=1e-5, atol=1e-6)
    np.testing.assert_array_equal(np.stack([host(t) for t in cq.x_q]), g[tag + "_lhs_xq"])


# ------------------------------------------------------------------ round 2: a15 ChannelQuantAct
def test_channel_quant_act_golden(K, golden):
    """a15 ChannelQuantAct 'none' (channelQuantAct.py:36-67) at shiftedScale 1, 33/32,
    31/32, 1/2: bit-exact q/dq with the [0, n-1] clamp (negatives and large values in the
    input hit both edges); torch.round has no gradient wrt x (d/dx == 0 exactly); the
    delta / zero_point gradients of the reference's autograd within 1e-5 (reductions)."""
    from shiftedscalequantization_amd import quant as Q
    g = golden("act_quant")
    x = dev(g["x"])
    uaq = Q.UniformAffineQuantizer(n_bits=4, channel_wise=False, scale_method="mse", leaf_param=True)
    uaq.delta = torch.nn.Parameter(dev(g["delta"]).view(()))
    uaq.zero_point = torch.nn.Parameter(dev(g["zp"]).view(()))
    uaq.inited = True
    for k, s in enumerate(g["scales"]):
        q = Q.ChannelQuantAct(uaq=uaq, shiftTarget=[1.0, 0.5])
        q.shiftedScale = float(s)
        xr = x.clone().requires_grad_(True)
        uaq.delta.grad = uaq.zero_point.grad = None
        y = q(xr)
        np.testing.assert_array_equal(host(y), g[f"s{k}_y"], err_msg=f"scale {s}")
        (y * dev(g[f"s{k}_gy"])).sum().backward()
        np.testing.assert_array_equal(host(xr.grad), g[f"s{k}_gx"])
        close(host(uaq.delta.grad).reshape(-1), g[f"s{k}_gdelta"], rtol=1e-5, atol=1e-5)
        close(host(uaq.zero_point.grad).reshape(-1), g[f"s{k}_gzp"], rtol=1e-5, atol=1e-5)
    hi = (2 ** 4 - 1 - float(g["zp"][0])) * float(g["delta"][0])
    assert host(y).min() >= -float(g["zp"][0]) * float(g["delta"][0]) * 0.5 - 1e-6
    assert host(q(x)).max() <= hi + 1e-6


# ------------------------------------------------------------------ round 2: prepared adaShift
# (256, 64, 3, 3) and (200, 37, 3, 3): the alpha backward's per-channel form in two load
# batches (Co*K 1281-2304), the latter with Ci not a multiple of the 8 XCDs (xcd_channel)
PREP_SHAPES = [(8, 6, 3, 3), (64, 64, 3, 3), (96, 48, 3, 3), (128, 64, 1, 1), (33, 5, 5, 5),
               (24, 1, 3, 3), (512, 512, 3, 3), (256, 128, 1, 1), (7, 300, 1, 1),
               (256, 64, 3, 3), (200, 37, 3, 3)]


@pytest.mark.parametrize("shape", PREP_SHAPES)
@pytest.mark.parametrize("S", [1, 2, 3, 4])
def test_adashift_prepared_matches_recompute(K, shape, S):
    """The prepared path (packed int8 floors + h(beta), one-launch alpha backward) gives
    the recomputing kernels' What bit for bit (soft and hard targets, soft and hard
    rounding) and their alpha gradients (+ fused regulariser from the device pair) to
    1e-6; repeated backward launches are bit-identical (fixed-order reduction)."""
    shifts = [31 / 32, 33 / 32, 1.0, 17 / 16][:S]
    gen = torch.Generator().manual_seed(hash((shape, S)) & 0xffff)
    w = torch.randn(shape, generator=gen) * 0.05
    d, z, _ = R.init_scale(w.numpy(), 2, False, True, "max")
    wd, dd, zd = w.cuda(), dev(d), dev(z)
    alpha, beta, _ = K.shift_init(wd, dd, shifts)
    alpha = alpha + torch.randn(alpha.shape, generator=gen).cuda() * 0.5
    if shape[1] == 1:
        alpha = alpha.view(1, -1)
    gy = torch.randn(shape, generator=gen).cuda()
    for hr in (0, 1):
        prep = K.AdaShiftPrep(wd, beta, dd, shifts, hr)
        assert prep.ok
        for ht in (0, 1):
            ref = K.adashift(alpha, beta, wd, dd, zd, shifts, 2, False, ht, hr)
            got = K.adashift_prepared(alpha, prep, dd, zd, 2, False, ht)
            np.testing.assert_array_equal(host(got), host(ref), err_msg=f"ht{ht} hr{hr}")
        regp = dev([0.1, 7.5])
        vals_ref = torch.zeros(alpha.numel() // S, device="cuda")
        vals_got = torch.zeros_like(vals_ref)
        a1 = alpha.clone().requires_grad_(True)
        K.adashift(a1, beta, wd, dd, zd, shifts, 2, False, 0, hr,
                   reg=(0.0, 0.0, vals_ref, regp)).backward(gy)
        grads = []
        for _ in range(3):
            a2 = alpha.clone().requires_grad_(True)
            vals_got.zero_()
            K.adashift_prepared(a2, prep, dd, zd, 2, False, 0,
                                reg=(0.0, 0.0, vals_got, regp)).backward(gy)
            grads.append(host(a2.grad))
        close(grads[0], host(a1.grad), rtol=1e-6, atol=1e-7)
        close(host(vals_got), host(vals_ref), rtol=1e-6, atol=1e-7)
        np.testing.assert_array_equal(grads[0], grads[1])
        np.testing.assert_array_equal(grads[0], grads[2])


def test_adashift_prepared_multi_equals_single(K):
    """Several weights in ONE multi-segment launch (a block's convs, up to 8 per launch and
    more in further launches) give each weight's single-launch What and alpha gradient
    bit for bit, with per-weight regulariser values."""
    shapes = [(64, 64, 3, 3), (128, 64, 3, 3), (128, 64, 1, 1), (7, 300, 1, 1), (24, 1, 3, 3),
              (33, 5, 5, 5), (96, 48, 3, 3), (512, 256, 3, 3), (16, 16, 3, 3), (40, 24, 1, 1),
              (256, 128, 3, 3), (256, 100, 1, 1)]
    gen = torch.Generator().manual_seed(11)
    regp = dev([0.1, 7.5])
    alphas, entries, gys, singles = [], [], [], []
    for k, shape in enumerate(shapes):
        w = torch.randn(shape, generator=gen) * 0.05
        d, z, _ = R.init_scale(w.numpy(), 2 if k % 2 else 4, False, True, "max")
        wd, dd, zd = w.cuda(), dev(d), dev(z)
        alpha, beta, _ = K.shift_init(wd, dd, SHIFTS)
        alpha = alpha + torch.randn(alpha.shape, generator=gen).cuda() * 0.5
        prep = K.AdaShiftPrep(wd, beta, dd, SHIFTS, 0)
        assert prep.ok
        bits = 2 if k % 2 else 4
        alphas.append(alpha)
        entries.append((prep, dd, zd, bits, False))
        gys.append(torch.randn(shape, generator=gen).cuda())
        a1 = alpha.clone().requires_grad_(True)
        v1 = torch.zeros(alpha.shape[0], device="cuda")
        y1 = K.adashift_prepared(a1, prep, dd, zd, bits, False, 0, reg=(0.0, 0.0, v1, regp))
        y1.backward(gys[-1])
        singles.append((host(y1), host(a1.grad), host(v1)))
    am = [a.clone().requires_grad_(True) for a in alphas]
    vals = [torch.zeros(a.shape[0], device="cuda") for a in alphas]
    ys = K.adashift_prepared_multi(am, entries, False, reg=(0.0, 0.0, vals, regp))
    torch.autograd.backward(list(ys), gys)
    for k, (y, a, v, (ys1, ga1, v1)) in enumerate(zip(ys, am, vals, singles)):
        np.testing.assert_array_equal(host(y), ys1, err_msg=str(shapes[k]))
        np.testing.assert_array_equal(host(a.grad), ga1, err_msg=str(shapes[k]))
        np.testing.assert_array_equal(host(v), v1, err_msg=str(shapes[k]))


def test_weights_qdq_ride_on_activation_qdq(K):
    """A deferred multi-tensor q/dq (K.deferred_fq_multi: per-channel W2 / W8 weights of
    several shapes, scalar-tail ones included) runs inside the next per-tensor q/dq launch:
    both outputs bit-identical to the separate launches; a table with no per-tensor launch
    after it is launched when the context ends."""
    gen = torch.Generator().manual_seed(9)
    act = torch.randn(7, 64, 56, 56, generator=gen).relu().cuda()
    d_a, z_a, _ = K.scale_init(act[:2], 4, False, False, "max")
    shapes = [(64, 3, 7, 7), (64, 64, 3, 3), (128, 64, 1, 1), (1000, 512), (33, 5, 3, 3)]
    ws, ds, zs, bits = [], [], [], []
    for k, shape in enumerate(shapes):
        w = (torch.randn(shape, generator=gen) * 0.05).cuda()
        b = 8 if k in (0, 3) else 2
        d, z, _ = K.scale_init(w, b, False, True, "max")
        ws.append(w), ds.append(d), zs.append(z), bits.append(b)
    ref_w = K.fake_quant_multi(ws, ds, zs, bits)
    ref_a, _ = K.fake_quant_fwd(act, d_a, z_a, 4)
    with K.deferred_fq_multi():
        got_w = K.fake_quant_multi(ws, ds, zs, bits)
        got_a, _ = K.fake_quant_fwd(act, d_a, z_a, 4)
    torch.cuda.synchronize()
    assert torch.equal(ref_a, got_a)
    for a, b in zip(ref_w, got_w):
        assert torch.equal(a, b)
    with K.deferred_fq_multi():
        late = K.fake_quant_multi(ws, ds, zs, bits)
    for a, b in zip(ref_w, late):
        assert torch.equal(a, b)


def test_prepared_forward_rides_on_gather(K):
    """A deferred prepared forward (K.deferred_prep_fwd) runs inside the next batch gather's
    launch: the What of every segment and the gathered rows are bit-identical to the two
    separate launches; a forward with no gather after it is launched when the context ends."""
    shapes = [(64, 64, 3, 3), (128, 64, 3, 3), (128, 64, 1, 1), (24, 5, 5, 5)]
    gen = torch.Generator().manual_seed(5)
    alphas, entries = [], []
    for shape in shapes:
        w = (torch.randn(shape, generator=gen) * 0.05).cuda()
        d, z, _ = K.scale_init(w, 2, False, True, "max")
        alpha, beta, _ = K.shift_init(w, d, SHIFTS)
        alphas.append(alpha + torch.randn(alpha.shape, generator=gen).cuda() * 0.5)
        entries.append((K.AdaShiftPrep(w, beta, d, SHIFTS, 0), d, z, 2, False))
    src0 = torch.randn(40, 3, 8, 9, generator=gen).cuda()      # rows of 216 floats (vec)
    src1 = torch.randn(40, 7, 5, generator=gen).cuda()         # rows of 35 floats (scalar)
    idx = torch.randperm(40, generator=gen)[:13].cuda()
    for s1 in (src0[:, :2], src1):
        ref_w = K.adashift_prepared_multi(alphas, entries, False)
        ref_g = K.gather_rows2(src0, idx, s1.contiguous())
        with K.deferred_prep_fwd():
            got_w = K.adashift_prepared_multi(alphas, entries, False)
            got_g = K.gather_rows2(src0, idx, s1.contiguous())
        torch.cuda.synchronize()
        for a, b in zip(ref_w, got_w):
            assert torch.equal(a, b)
        for a, b in zip(ref_g, got_g):
            assert torch.equal(a, b)
    with K.deferred_prep_fwd():
        late = K.adashift_prepared_multi(alphas, entries, False)
    for a, b in zip(ref_w, late):
        assert torch.equal(a, b)


def test_adashift_prepared_overflow_falls_back(K):
    """A floor outside int8 (an 8-bit weight with a tiny delta) marks the preparation
    unusable; ChannelQuant then keeps the recomputing kernels with identical results."""
    from shiftedscalequantization_amd import quant as Q
    w = torch.randn(16, 8, 3, 3).cuda() * 0.05
    d = torch.full((16, 1, 1, 1), 1e-4, device="cuda")
    beta = torch.zeros_like(w)
    prep = K.AdaShiftPrep(w, beta, d, SHIFTS, 0)
    assert not prep.ok
    uaq = Q.UniformAffineQuantizer(n_bits=8, channel_wise=True, ch=w.shape).cuda()
    uaq.delta = torch.nn.Parameter(d.clone())
    uaq.zero_point = torch.nn.Parameter(torch.full_like(d, 128.0))
    uaq.inited = True
    cq = Q.ChannelQuant(1.0, uaq=uaq, weight_tensor=w, shiftTarget=SHIFTS)
    cq.init_v_beta(w)
    cq.opt_mode = "adaShift"
    cq.beta.requires_grad_(False)
    y = cq(w)
    assert cq._prep is not None and cq._prep[1] is None
    ref = K.adashift(cq.alpha, cq.beta, w, cq.delta, cq.zero_point, SHIFTS, 8, False, 0, 0)
    np.testing.assert_array_equal(host(y), host(ref))


# ------------------------------------------------------------------ round 2: finalisation
@pytest.mark.parametrize("fixture", ["recon_fused", "recon_driver"])
def test_hard_weights_from_reference_alpha_bit_exact(K, golden, fixture):
    """a25: given the reference's FINAL alpha and beta, the finished quantizer (hard
    targets, hard rounding) reproduces the reference's hard What bit for bit, through the
    prepared kernel, the recomputing kernel and the export path's integer codes
    ((code - zp) * delta == What exactly)."""
    g = golden(fixture)
    if fixture == "recon_fused":
        items = [(n, g[n + "_w"], g[n + "_delta"], g[n + "_zp"], g[n + "_alpha"], g[n + "_beta0"],
                  g[n + "_what_hard"]) for n in ("conv1", "conv2", "downsample")]
    else:
        items = []
        qm = {1: ("b0", "conv1"), 2: ("b0", "conv2"), 3: ("b1", "conv1"), 4: ("b1", "conv2"),
              5: ("b1", "downsample")}
        for k, (b, n) in qm.items():
            items.append((f"{b}.{n}", g[f"qm{k}_w"], g[f"qm{k}_delta"], g[f"qm{k}_zp"],
                          g[f"{b}_{n}_alpha"], g[f"{b}_{n}_beta0"], g[f"{b}_{n}_what_hard"]))
    for name, w, d, z, alpha, beta, what in items:
        d4, z4 = dev(d).view(-1, 1, 1, 1), dev(z).view(-1, 1, 1, 1)
        y = K.adashift(dev(alpha), dev(beta), dev(w), d4, z4, SHIFTS, 2, False, 1, 1)
        np.testing.assert_array_equal(host(y), what, err_msg=name)
        prep = K.AdaShiftPrep(dev(w), dev(beta), d4, SHIFTS, 1)
        yp = K.adashift_prepared(dev(alpha), prep, d4, z4, 2, False, 1)
        np.testing.assert_array_equal(host(yp), what, err_msg=name)
        y2, codes = K.adashift_codes(dev(alpha), dev(beta), dev(w), d4, z4, SHIFTS, 2, False)
        c = codes.cpu().numpy().astype(np.float32)
        np.testing.assert_array_equal((c - z.reshape(-1, 1, 1, 1)) * d.reshape(-1, 1, 1, 1), what)


@pytest.mark.parametrize("resepi", [False, True])
@pytest.mark.parametrize("p", [2.0, 2.4])
@pytest.mark.parametrize("hw", [7, 8])
@pytest.mark.parametrize("quant", [False, True])
@pytest.mark.parametrize("relu", [0, 1])
def test_epilogue_loss_bwd_matches_separate_passes(K, hw, quant, relu, p, resepi):
    """ssq_epilogue_loss_bwd (the fused tail) vs the three passes it replaces -- epilogue
    forward, lp_loss_rows (p = 2: the shifted-scale loops; 2.4: BRECQ's act phase) against
    the cached target rows, epilogue backward -- on
    float4 rows (8x8) and scalar rows (7x7), with gamma^z/phi^z, a residual, ReLU or
    identity (InvertedResidual tails) and optionally the per-tensor act quantizer: every
    gradient bit-identical, the loss value to the last ulps (row vs block partials).
    resepi: the residual is a downsample branch whose own epilogue (bias, gamma^z/phi^z, no
    activation) the tail applies (K.LazyRes) instead of two more passes: dL/d(its conv
    output) and its gamma / phi gradients bit-identical too."""
    from shiftedscalequantization_amd.quant.quant_layer import UniformAffineQuantizer
    gen = torch.Generator().manual_seed(hw * 4 + int(quant) * 2 + relu)
    N, C = 6, 20
    y = torch.randn(N, C, hw, hw, generator=gen).cuda()
    res = torch.randn(N, C, hw, hw, generator=gen).cuda().requires_grad_(True)
    bias = torch.randn(C, generator=gen).cuda()
    gamma = (1 + 0.1 * torch.randn(1, C, 1, 1, generator=gen)).cuda().requires_grad_(True)
    phi = (0.1 * torch.randn(1, C, 1, 1, generator=gen)).cuda().requires_grad_(True)
    cache = torch.randn(15, C, hw, hw, generator=gen).relu().cuda()
    idx = torch.tensor([3, 14, 0, 7, 7, 9], dtype=torch.int64).cuda()
    if resepi:
        yds = torch.randn(N, C, hw, hw, generator=gen).cuda().requires_grad_(True)
        bds = torch.randn(C, generator=gen).cuda()
        gds = (1 + 0.1 * torch.randn(1, C, 1, 1, generator=gen)).cuda().requires_grad_(True)
        pds = (0.1 * torch.randn(1, C, 1, 1, generator=gen)).cuda().requires_grad_(True)
    q = None
    if quant:
        q = UniformAffineQuantizer(n_bits=4, channel_wise=False, scale_method="max", leaf_param=True).cuda()
        q.delta = torch.nn.Parameter(torch.tensor(0.21).cuda())
        q.zero_point = torch.nn.Parameter(torch.tensor(0.0).cuda())
        q.inited = True
    # separate passes
    yr = y.clone().requires_grad_(True)
    res_in = K.epilogue(yds, bds, gds, pds, None, 0, None) if resepi else res
    out = K.epilogue(yr, bias, gamma, phi, res_in, relu, q)
    loss1, g1 = K.lp_loss_and_grad(out, K.Rows(cache, idx), p)
    out.backward(g1)
    sep = [yr.grad, yds.grad if resepi else res.grad, gamma.grad, phi.grad] + \
        ([q.delta.grad, q.zero_point.grad] if quant else []) + ([gds.grad, pds.grad] if resepi else [])
    sep = [host(t).copy() for t in sep]
    for t in [res, gamma, phi] + ([q.delta, q.zero_point] if quant else []) + \
            ([yds, gds, pds] if resepi else []):
        t.grad = None
    if resepi:
        res = K.LazyRes(yds, bds, gds, pds)
    # fused
    # the lazy placeholder carries exactly these inputs (taken on float4 rows, and on
    # scalar rows while K.TAIL_SCALAR is set)
    lazy = K.epilogue(y, bias, gamma, phi, res, relu, q, lazy=True)
    assert hasattr(lazy, "_ssq_tail") == (hw * hw % 4 == 0 or K.TAIL_SCALAR)
    tail = (y, bias, gamma, phi, res, relu, q)
    loss2, gy, gres, ggm, gph, gd, gz, grg, grph = K.epilogue_loss_bwd(tail, K.Rows(cache, idx),
                                                                        N * hw * hw, p)
    fused = [gy, gres, ggm, gph] + ([gd, gz] if quant else []) + ([grg, grph] if resepi else [])
    for a, b in zip(sep, fused):
        np.testing.assert_array_equal(a.reshape(-1).view(np.int32), host(b).reshape(-1).view(np.int32))
    close(host(loss2), host(loss1), rtol=1e-6, atol=0)


@pytest.mark.parametrize("quant", [False, True])
def test_epilogue_bwd_without_dy(K, quant):
    """The epilogue backward of a frozen conv (dL/dy not wanted: BRECQ's act phase) writes no
    gy and still produces the gamma^z / phi^z / delta / zero-point sums bit-identical to the
    pass that does write gy."""
    from shiftedscalequantization_amd.quant.quant_layer import UniformAffineQuantizer
    gen = torch.Generator().manual_seed(11 + int(quant))
    N, C, hw = 4, 12, 8
    y = torch.randn(N, C, hw, hw, generator=gen).cuda()
    bias = torch.randn(C, generator=gen).cuda()
    g = torch.randn(N, C, hw, hw, generator=gen).cuda()
    runs = []
    for need_dy in (True, False):
        gamma = (1 + 0.1 * torch.randn(1, C, 1, 1, generator=torch.Generator().manual_seed(3))).cuda().requires_grad_(True)
        phi = (0.1 * torch.randn(1, C, 1, 1, generator=torch.Generator().manual_seed(4))).cuda().requires_grad_(True)
        q = None
        if quant:
            q = UniformAffineQuantizer(n_bits=4, channel_wise=False, scale_method="max", leaf_param=True).cuda()
            q.delta = torch.nn.Parameter(torch.tensor(0.19).cuda())
            q.zero_point = torch.nn.Parameter(torch.tensor(1.0).cuda())
            q.inited = True
        yr = y.clone().requires_grad_(need_dy)
        out = K.epilogue(yr, bias, gamma, phi, None, 1, q)
        out.backward(g)
        assert (yr.grad is not None) == need_dy
        got = [gamma.grad, phi.grad] + ([q.delta.grad, q.zero_point.grad] if quant else [])
        runs.append([host(t).reshape(-1).view(np.int32).copy() for t in got])
    for a, b in zip(*runs):
        np.testing.assert_array_equal(a, b)


@pytest.mark.parametrize("form", ["affine_q", "bias_q", "bias_act"])
@pytest.mark.parametrize("hw", [7, 8])
def test_epilogue_rows_in_place_bit_identical(K, hw, form):
    """ssq_epilogue_*_rows (BRECQ's act phase, block_recon.ROWS_IN_PLACE): the K13 epilogue
    forward and backward reading a frozen conv's output rows in place from its per-sample
    cache by the batch indices (duplicates included), and the fused tail reading the
    residual's rows in place, against the same calls on the gathered batch -- outputs and
    every gradient bit-identical, nothing gathered behind the call (no fptr fallback); the
    forwards take a row-view residual too (the non-fused block tail of the act phase).
    Forms: the --bias_cal affine epilogue + act quantizer (EpilogueFn), bias + ReLU + act
    quantizer (BiasActQuantFn), bias + ReLU (BiasActFn); float4 rows (8x8), scalar (7x7)."""
    from shiftedscalequantization_amd import _capi as A
    from shiftedscalequantization_amd.quant.quant_layer import UniformAffineQuantizer
    gen = torch.Generator().manual_seed(hw * 3 + len(form))
    C = 12
    cache = torch.randn(9, C, hw, hw, generator=gen).cuda()
    rcache = torch.randn(9, C, hw, hw, generator=gen).cuda()
    tcache = torch.randn(9, C, hw, hw, generator=gen).relu().cuda()
    idx = torch.tensor([4, 1, 8, 1, 0], dtype=torch.int64).cuda()
    N = idx.numel()
    bias = torch.randn(C, generator=gen).cuda()
    g = torch.randn(N, C, hw, hw, generator=gen).cuda()
    y2 = torch.randn(N, C, hw, hw, generator=gen).cuda()     # the tail's conv output

    def quantizer():
        q = UniformAffineQuantizer(n_bits=4, channel_wise=False, scale_method="max", leaf_param=True).cuda()
        q.delta = torch.nn.Parameter(torch.tensor(0.23).cuda())
        q.zero_point = torch.nn.Parameter(torch.tensor(2.0).cuda())
        q.inited = True
        return q

    def run(view):
        gm = (1 + 0.1 * torch.randn(1, C, 1, 1, generator=torch.Generator().manual_seed(5))).cuda().requires_grad_(True)
        ph = (0.1 * torch.randn(1, C, 1, 1, generator=torch.Generator().manual_seed(6))).cuda().requires_grad_(True)
        q = quantizer()
        falls = []
        orig = A.materialize_rows

        def mat(t):
            if t.data_ptr() in A.ROW_VIEWS:
                falls.append(1)
            return orig(t)

        A.materialize_rows = mat
        try:
            with K.row_views():
                yb = torch.empty(N, C, hw, hw, device="cuda")
                rb = torch.empty(N, C, hw, hw, device="cuda")
                if view:
                    K.rows_view(yb, cache, idx)
                    K.rows_view(rb, rcache, idx)
                else:
                    yb.copy_(cache[idx])
                    rb.copy_(rcache[idx])
                if form == "affine_q":
                    out = K.epilogue(yb, bias, gm, ph, rb, 1, q)
                elif form == "bias_q":
                    out = K.bias_act_quant(yb, bias, rb, 1, q.delta, q.zero_point, 4)
                else:
                    gm = ph = None
                    out = K.bias_act(yb, bias, rb, 1)
                res_out = [host(out).copy()]
                if out.requires_grad:
                    out.backward(g)
                    res_out += [host(t).copy() for t in (gm, ph) if t is not None]
                    if form != "bias_act":
                        res_out += [host(q.delta.grad).copy(), host(q.zero_point.grad).copy()]
                # the fused tail with the residual read in place (its rows' gradient wanted)
                tail = (y2, bias, None, None, rb, 1, None)
                loss, gy, gres = K.epilogue_loss_bwd(tail, K.Rows(tcache, idx), N * hw * hw, 2.4)[:3]
                res_out += [host(loss).copy(), host(gy).copy()]
        finally:
            A.materialize_rows = orig
        return res_out, falls

    (a, fa), (b, fb) = run(False), run(True)
    assert not fb and len(a) == len(b)
    for u, v in zip(a, b):
        np.testing.assert_array_equal(u.reshape(-1).view(np.int32), v.reshape(-1).view(np.int32))


@pytest.mark.parametrize("shape", [(8, 125, 5), (11, 100, 8), (40, 500, 7)])
def test_epilogue_bwd_delta_split(K, shape):
    """The act quantizer's delta / zero-point sums of the epilogue backward over many rows:
    one workgroup per 1024 rows (<= 16), the last to arrive adding the partials in range
    order (csrc/fin_tasks.h fin_epi).  1000 rows (one workgroup), 1100 (two), 20000 (16).
    Against the float64 sum of the launch's own row records; deferred (riding on a later
    launch) and standalone bit-identical; repeated calls identical (the counter resets); and
    the unfused epilogue + fake-quant composition within the affine epilogue's tolerance."""
    from shiftedscalequantization_amd import _capi as A
    from shiftedscalequantization_amd.quant.quant_layer import UniformAffineQuantizer
    N, C, hw = shape
    gen = torch.Generator().manual_seed(N + C)
    y = torch.randn(N, C, hw, hw, generator=gen).cuda()
    bias = (0.1 * torch.randn(C, generator=gen)).cuda()
    g = torch.randn(N, C, hw, hw, generator=gen).cuda()
    gm0 = (1 + 0.1 * torch.randn(1, C, 1, 1, generator=gen)).cuda()
    ph0 = (0.1 * torch.randn(1, C, 1, 1, generator=gen)).cuda()

    def run(defer, fused=True):
        gamma, phi = gm0.clone().requires_grad_(True), ph0.clone().requires_grad_(True)
        q = UniformAffineQuantizer(n_bits=4, channel_wise=False, scale_method="max", leaf_param=True).cuda()
        q.delta = torch.nn.Parameter(torch.tensor(0.23).cuda())
        q.zero_point = torch.nn.Parameter(torch.tensor(3.0).cuda())
        q.inited = True
        cache = {}
        with A.workspace_scope(cache), K.deferred_finalize(defer):
            if fused:
                out = K.epilogue(y, bias, gamma, phi, None, 1, q)
            else:
                out = q(K.epilogue(y, bias, gamma, phi, None, 1, None))
            out.backward(g)
        torch.cuda.synchronize()
        ws = [b for k, b in cache.items() if k[2] == K._epi_slot_name()] if fused else []
        return [host(t).reshape(-1).copy() for t in (q.delta.grad, q.zero_point.grad, gamma.grad,
                                                     phi.grad)], ws

    base, ws = run(False)
    rows = N * C
    rec = ws[0][:rows * 9 * 8].view(torch.float64).view(rows, 9).cpu().numpy()
    a = rec[:, 2:6].sum(axis=0)
    np.testing.assert_allclose(base[0], [a[0] - a[1]], rtol=1e-6, atol=0)
    np.testing.assert_allclose(base[1], [a[2] - a[3]], rtol=1e-6, atol=1e-6)
    for defer in (True, False, True):
        got, _ = run(defer)
        for x, b in zip(got, base):
            np.testing.assert_array_equal(x.view(np.int32), b.view(np.int32))
    unf, _ = run(False, fused=False)
    # delta / zp: the same (x/d)/d terms in two double summation orders (see
    # _compare_fused_unfused); gamma / phi: double vs torch's fp32 sums
    for k, (x, b) in enumerate(zip(base, unf)):
        if k < 2:
            np.testing.assert_allclose(x, b, rtol=1e-6, atol=1e-6 * max(1.0, float(np.abs(b).max())))
        else:
            np.testing.assert_allclose(x, b, rtol=1e-4, atol=1e-3 * max(1.0, float(np.abs(b).max())))


@pytest.mark.parametrize("defer", [False, True])
def test_epilogue_bwd_delta_split_two_streams(K, defer):
    """The delta reduction's last-arriver counter lives in each call's workspace
    (fin_tasks.h delta_ticket_offset), so epilogue backwards running at the same time on two
    streams (20000 rows each: 16 delta workgroups apiece) cannot count each other's
    workgroups: every gradient equals the one-stream result bit for bit."""
    from shiftedscalequantization_amd import _capi as A
    from shiftedscalequantization_amd.quant.quant_layer import UniformAffineQuantizer
    N, C, hw = 40, 500, 7
    gen = torch.Generator().manual_seed(4242)
    ys = [torch.randn(N, C, hw, hw, generator=gen).cuda() for _ in range(2)]
    gs = [torch.randn(N, C, hw, hw, generator=gen).cuda() for _ in range(2)]
    bias = (0.1 * torch.randn(C, generator=gen)).cuda()
    gm0 = (1 + 0.1 * torch.randn(1, C, 1, 1, generator=gen)).cuda()
    ph0 = (0.1 * torch.randn(1, C, 1, 1, generator=gen)).cuda()

    def launch(i):
        gamma, phi = gm0.clone().requires_grad_(True), ph0.clone().requires_grad_(True)
        q = UniformAffineQuantizer(n_bits=4, channel_wise=False, scale_method="max", leaf_param=True).cuda()
        q.delta = torch.nn.Parameter(torch.tensor(0.23).cuda())
        q.zero_point = torch.nn.Parameter(torch.tensor(3.0).cuda())
        q.inited = True
        with A.workspace_scope({}), K.deferred_finalize(defer):
            out = K.epilogue(ys[i], bias, gamma, phi, None, 1, q)
            out.backward(gs[i])
        return q, gamma, phi

    def grads(r):
        q, gamma, phi = r
        return [host(t).reshape(-1).view(np.int32).copy()
                for t in (q.delta.grad, q.zero_point.grad, gamma.grad, phi.grad)]

    base = []
    for i in range(2):
        r = launch(i)
        torch.cuda.synchronize()
        base.append(grads(r))
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    for _ in range(8):
        res = []
        for i in range(2):
            with torch.cuda.stream(streams[i]):
                res.append(launch(i))
        torch.cuda.synchronize()
        for i in range(2):
            for x, b in zip(grads(res[i]), base[i]):
                np.testing.assert_array_equal(x, b)


@pytest.mark.parametrize("defer", [False, True])
def test_lp_loss_two_streams(K, defer):
    """ssq_lp_loss keeps no device-global state (its one-launch form and the counter it
    needed are gone): the partials live in the call's workspace, one per stream, so two loss
    passes in flight on two streams -- standalone finalize or finalize tasks queued on each
    stream and flushed there -- give the one-stream values and gradients bit for bit, and the
    value is the float64 loss to 1e-6."""
    from shiftedscalequantization_amd import _capi as A
    gen = torch.Generator().manual_seed(77)
    # 1024 workgroups apiece (the launch's cap): both grids fill the chip together
    preds = [torch.randn(64, 256, 28, 28, generator=gen).cuda() for _ in range(2)]
    tgts = [torch.randn(64, 256, 28, 28, generator=gen).cuda() for _ in range(2)]

    def run(i, p):
        with K.deferred_finalize(defer):
            loss, g = K.lp_loss_and_grad(preds[i], tgts[i], p)
        return loss, g

    def bits(r):
        return [host(t).reshape(-1).view(np.int32).copy() for t in r]

    for p in (2.0, 2.4):
        base = []
        for i in range(2):
            r = run(i, p)
            torch.cuda.synchronize()
            base.append(bits(r))
        streams = [torch.cuda.Stream(), torch.cuda.Stream()]
        for _ in range(8):
            res = []
            for i in range(2):
                with torch.cuda.stream(streams[i]), A.workspace_scope({}):
                    res.append(run(i, p))
            torch.cuda.synchronize()
            for i in range(2):
                for a, b in zip(bits(res[i]), base[i]):
                    np.testing.assert_array_equal(a, b)
        if p == 2.0:
            for i in range(2):
                ref = (preds[i] - tgts[i]).double().abs().pow(p).sum(1).mean().item()
                got = float(base[i][0].view(np.float32)[0])
                assert abs(got - ref) <= 1e-6 * abs(ref), (got, ref)


@pytest.mark.parametrize("bs,Co,Ci,lam", [(32, 1000, 512, 0.01), (8, 10, 64, 0.0), (64, 37, 320, 0.01),
                                          (33, 70, 256, 0.01), (1, 16, 4096, 0.01)])
def test_fc_recon_iter_vs_reference(K, bs, Co, Ci, lam):
    """K19 ssq_fc_recon_iter, one iteration against its parts: the loss and dL/dy against the
    float64 evaluation of x[idx] W^T + bias with W^ the AdaRound forward (bit-exact kernel);
    V's gradient against ssq_adaround_bwd fed the float64 dW (fp32 rounding); V's Adam step
    bit-identical to ssq_adam applied to the fused kernel's own V gradient."""
    gen = torch.Generator().manual_seed(bs + Co)
    N = 3 * bs
    x = torch.relu(torch.randn(N, Ci, generator=gen)).cuda()
    tgt = torch.randn(N, Co, generator=gen).cuda()
    w = (0.05 * torch.randn(Co, Ci, generator=gen)).cuda()
    bias = (0.1 * torch.randn(Co, generator=gen)).cuda()
    d, z, _ = K.scale_init(w, 8, False, True, "max")
    v = K.rect_init(w, d)
    v += (0.3 * torch.randn(Co, Ci, generator=gen)).cuda()
    m = (1e-3 * torch.randn(Co, Ci, generator=gen)).cuda()
    s2 = (1e-6 * torch.rand(Co, Ci, generator=gen)).cuda()
    idx = torch.randperm(N, generator=gen)[:bs]
    slot = torch.zeros(bs + 2, dtype=torch.int64)
    slot[:bs] = idx
    words = np.array([lam, 12.5, -1e-3 / (1 - 0.9 ** 7), (1 - 0.999 ** 7) ** 0.5], np.float32)
    slot[bs:] = torch.from_numpy(words.view(np.int64))
    slot = slot.cuda()
    v0, m0, s0 = v.clone(), m.clone(), s2.clone()
    gv = torch.empty_like(v)
    what_in = K.adaround(v0, w, d, z, 8, False, False).detach().clone()
    what_buf = what_in.clone()
    loss, g = K.fc_recon_iter(x, tgt, slot, bs, w, v, what_buf, d, z, 8, bias, m, s2, 0.9, 0.999,
                              1e-8, gv_out=gv)
    torch.cuda.synchronize()
    # the next iteration's W^: ssq_adaround_fwd of the updated V, bit for bit
    np.testing.assert_array_equal(host(what_buf).view(np.int32),
                                  host(K.adaround(v, w, d, z, 8, False, False)).view(np.int32))
    # float64 truth of the forward / loss / gradient
    what = what_in.double()
    xb, tb = x[idx.cuda()].double(), tgt[idx.cuda()].double()
    y = xb @ what.t() + bias.double()
    ref_loss = ((y - tb) ** 2).sum(1).mean().item()
    ref_g = 2.0 * (y - tb) / bs
    assert abs(loss.item() - ref_loss) <= 1e-5 * abs(ref_loss)
    np.testing.assert_allclose(host(g), ref_g.cpu().numpy(), rtol=0, atol=1e-5 * ref_g.abs().max().item())
    # V's gradient: ssq_adaround_bwd with the rounding regulariser, on the float64 dW
    dw = (ref_g.t() @ xb).float()
    regp = torch.tensor(words[:2]).cuda()
    vv = v0.clone().requires_grad_(True)
    K.adaround(vv, w, d, z, 8, False, False, reg=(0.0, 0.0, regp)).backward(dw)
    gref = host(vv.grad)
    scale = np.abs(gref).max()
    assert np.max(np.abs(host(gv) - gref)) <= 1e-4 * scale
    # Adam on the kernel's own gradient: ssq_adam's bits
    vr, mr, sr = v0.clone(), m0.clone(), s0.clone()
    K.adam_step([vr], [gv], [mr], [sr], 0.9, 0.999, 1e-8, hyper=torch.tensor(words[2:]).cuda())
    for a, b in ((v, vr), (m, mr), (s2, sr)):
        np.testing.assert_array_equal(host(a).view(np.int32), host(b).view(np.int32))


def test_armed_adam_falls_back_when_not_covered(K):
    """An armed step the alpha backward cannot take entirely (a parameter whose gradient
    no launch of the stream produced) is left alone: adam_take() is False and nothing was
    updated by the launch."""
    w = (torch.randn(64, 64, 3, 3) * 0.05).cuda()
    d, z, _ = K.scale_init(w, 2, False, True, "max")
    alpha, beta, _ = K.shift_init(w, d, [31 / 32, 33 / 32, 1.0])
    prep = K.AdaShiftPrep(w, beta, d, [31 / 32, 33 / 32, 1.0], 0)
    a = alpha.clone().requires_grad_(True)
    other = torch.zeros(10, device="cuda")
    ms = [torch.zeros_like(a), torch.zeros_like(other)]
    vs = [torch.zeros_like(a), torch.zeros_like(other)]
    hyper = torch.tensor([-1e-3, 0.5], device="cuda")
    K.adam_arm([a, other], ms, vs, 0.9, 0.999, 1e-8, hyper)
    y = K.adashift_prepared(a, prep, d, z, 2, False, 0)
    y.backward(torch.randn_like(y))
    torch.cuda.synchronize()
    assert not K.adam_take()
    assert torch.equal(a.detach(), alpha) and not torch.any(ms[0] != 0)
    # armed on the launch's own alpha only: taken, and the update is ssq_adam's
    b = alpha.clone().requires_grad_(True)
    m1, v1 = torch.zeros_like(b), torch.zeros_like(b)
    K.adam_arm([b], [m1], [v1], 0.9, 0.999, 1e-8, hyper)
    gy = torch.randn_like(y)
    K.adashift_prepared(b, prep, d, z, 2, False, 0).backward(gy)
    torch.cuda.synchronize()
    assert K.adam_take()
    c = alpha.clone().requires_grad_(True)
    m2, v2 = torch.zeros_like(c), torch.zeros_like(c)
    K.adashift_prepared(c, prep, d, z, 2, False, 0).backward(gy)
    with torch.no_grad():
        K.adam_step([c], [c.grad], [m2], [v2], 0.9, 0.999, 1e-8, hyper=hyper)
    assert torch.equal(b.grad, c.grad)
    assert torch.equal(b.detach(), c.detach()) and torch.equal(m1, m2) and torch.equal(v1, v2)
