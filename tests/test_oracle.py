"""Pin the CPU oracle (oracle/ssq_ref.py) to the reference's own outputs (tests/golden).

Integer codes / exact fp32 dequant values must match bit-exactly; values that pass
through a transcendental (softmax, sigmoid, log, pow) or a reduction are held to a
relative tolerance (the reference's summation order and libm are not reproducible).
"""
import numpy as np
import pytest

from oracle import ssq_ref as R

RTOL = 1e-5


def close(a, b, rtol=RTOL, atol=1e-6):
    np.testing.assert_allclose(np.asarray(a, np.float64), np.asarray(b, np.float64), rtol=rtol, atol=atol)


def tags(g, suffix):
    return sorted(k[: -len(suffix)] for k in g if k.endswith(suffix))


# ------------------------------------------------------------------ UAQ (K1-K4)
def test_uaq_init_and_forward_bit_exact(golden):
    g = golden("uaq")
    seen = 0
    for t in tags(g, "_delta"):
        if t == "zero":
            continue
        bits = int(t.split("_")[0][1:])
        sym = "_sym_" in t
        cw = "_cw_" in t
        method = t.rsplit("_", 1)[1]
        x = g[t + "_x"]
        d, z, r = R.init_scale(x, bits, sym, cw, method)
        np.testing.assert_array_equal(np.asarray(d).reshape(-1), g[t + "_delta"], err_msg=t)
        np.testing.assert_array_equal(np.asarray(z).reshape(-1), g[t + "_zp"], err_msg=t)
        y, _ = R.fake_quant(x, d, z, bits, sym)
        np.testing.assert_array_equal(y, g[t + "_y"], err_msg=t)
        seen += 1
    assert seen >= 16


def test_uaq_zero_range_channel(golden):
    g = golden("uaq")
    d, z, _ = R.init_scale(g["zero_x"], 2, False, True, "max")
    np.testing.assert_array_equal(d.reshape(-1), g["zero_delta"])
    assert d.reshape(-1)[0] == np.float32(1e-8)
    y, _ = R.fake_quant(g["zero_x"], d, z, 2)
    np.testing.assert_array_equal(y, g["zero_y"])


def _init_case(d, tag):
    method, cw, sym = tag.split("_")[:3]
    return d[tag + "_x"], method, cw == "cw", sym == "sym", int(d[tag + "_status"][0])


def test_init_specials(golden):
    """init_quantization_scale with NaN / +-inf / 3e38 / constant / zero rows planted BEFORE
    the init (quant_layer.py:100-166): where the reference returns a scale the oracle's is
    bit-identical; where it raises, the oracle raises the same exception type; where it
    returns None (per-tensor 'mse'), so does the oracle."""
    d = golden("init_specials")
    for tag in d["cases"]:
        x, method, cw, sym, status = _init_case(d, tag)
        if status == 1:
            exc = {"ValueError": ValueError, "TypeError": TypeError}[str(d[tag + "_exc"][0])]
            with pytest.raises(exc):
                R.init_scale(x, 4, sym, cw, method)
            continue
        dl, zp, rz = R.init_scale(x, 4, sym, cw, method)
        if status == 2:
            assert dl is None, tag
            continue
        np.testing.assert_array_equal(np.ravel(dl), d[tag + "_delta"], err_msg=tag)
        np.testing.assert_array_equal(np.ravel(zp), d[tag + "_zp"], err_msg=tag)
        np.testing.assert_array_equal(np.ravel(rz), d[tag + "_rawzp"], err_msg=tag)


def test_uaq_backward(golden):
    g = golden("uaq")
    for t in tags(g, "_gdelta"):
        bits = int(t.split("_")[0][1:])
        sym = "_sym_" in t
        x = g[t + "_x"]
        shape = (-1,) + (1,) * (x.ndim - 1) if "_cw_" in t else ()
        d = g[t + "_delta"].reshape(shape)
        z = g[t + "_zp"].reshape(shape)
        gx, gd, gz = R.fake_quant_bwd(x, d, z, bits, sym, g[t + "_gy"])
        np.testing.assert_array_equal(gx, g[t + "_gx"], err_msg=t)
        close(np.reshape(gd, -1), g[t + "_gdelta"], rtol=1e-4, atol=1e-4)
        close(np.reshape(gz, -1), g[t + "_gzp"], rtol=1e-4, atol=1e-4)


def test_uaq_specials(golden):
    """NaN / +-inf / +-0 / +-3e38 inputs (uaq_specials.npz): NaN where the reference gives
    NaN (torch.clamp keeps NaN; round_ste turns an infinite x/delta into NaN), every other
    value bit for bit; ChannelQuantAct 'none' (torch.round) clamps +-inf to an edge."""
    g = golden("uaq_specials")
    for t in tags(g, "_gdelta"):
        if t.startswith("act_"):
            continue
        bits = int(t.split("_")[0][1:])
        sym = "_sym_" in t
        x = g[t + "_x"]
        shape = (-1,) + (1,) * (x.ndim - 1) if "_cw_" in t else ()
        d, z = g[t + "_delta"].reshape(shape), g[t + "_zp"].reshape(shape)
        y, _ = R.fake_quant(x, d, z, bits, sym)
        np.testing.assert_array_equal(y, g[t + "_y"], err_msg=t)
        assert np.isnan(y).sum() > np.isnan(x).sum(), t          # the infinities too
        gx, gd, gz = R.fake_quant_bwd(x, d, z, bits, sym, g[t + "_gy"])
        np.testing.assert_array_equal(gx, g[t + "_gx"], err_msg=t)
        close(np.reshape(gd, -1), g[t + "_gdelta"], rtol=1e-4, atol=1e-4)
        close(np.reshape(gz, -1), g[t + "_gzp"], rtol=1e-4, atol=1e-4)
    x = g["b4_asym_pt_mse_x"]
    for k in (0, 1):
        sc = float(g[f"act_s{k}_scale"][0])
        d = np.float32(g["b4_asym_pt_mse_delta"][0]) * np.float32(sc)
        y, _ = R.fake_quant(x, d, g["b4_asym_pt_mse_zp"][0], 4, False, ste=False)
        np.testing.assert_array_equal(y, g[f"act_s{k}_y"])
        assert np.isnan(y).sum() == np.isnan(x).sum()


# ------------------------------------------------------------------ ChannelQuant (K5-K9)
SHIFTS = [31 / 32, 33 / 32, 1.0]


def _cq_setup(g, tag):
    w = g[tag + "_w"]
    is_fc = w.ndim != 4
    shape = (-1, 1) if is_fc else (-1, 1, 1, 1)
    d = g[tag + "_delta"].reshape(shape)
    z = g[tag + "_zp"].reshape(shape)
    bits = int(tag.rsplit("_b", 1)[1])
    return w, is_fc, d, z, bits


CQ_FILES = ["channelquant", "channelquant_specials"]   # _specials: NaN / +-inf / +-0 in W


@pytest.mark.parametrize("fname", CQ_FILES)
@pytest.mark.parametrize("tag", ["conv_b2", "conv_b4", "fc_b2", "fc_b4", "dw_b2", "dw_b4"])
def test_channelquant_init_v_beta(golden, tag, fname):
    g = golden(fname)
    w, is_fc, d, z, bits = _cq_setup(g, tag)
    xq, alpha, beta = R.init_v_beta(w, d, SHIFTS)
    np.testing.assert_array_equal(np.stack(xq), g[tag + "_xq"])
    close(alpha, g[tag + "_alpha0"])
    close(beta, g[tag + "_beta"], rtol=1e-5, atol=1e-5)
    # hard-round decisions derived from beta are exact
    np.testing.assert_array_equal(beta >= 0, g[tag + "_beta"] >= 0)


@pytest.mark.parametrize("fname", CQ_FILES)
@pytest.mark.parametrize("tag", ["conv_b2", "conv_b4", "fc_b2", "fc_b4", "dw_b2", "dw_b4"])
def test_channelquant_adashift(golden, tag, fname):
    g = golden(fname)
    w, is_fc, d, z, bits = _cq_setup(g, tag)
    xq = list(g[tag + "_xq"])
    alpha, beta = g[tag + "_alpha"], g[tag + "_beta"]
    close(R.sig_soft_targets(alpha), g[tag + "_p"])
    close(R.soft_round(beta), g[tag + "_h"])
    np.testing.assert_array_equal(R.get_delta(d, alpha, SHIFTS, is_fc), g[tag + "_delta_sel"])
    for ht, hr in ((0, 0), (1, 1), (0, 1), (1, 0)):
        k = f"{tag}_t{ht}r{hr}"
        y = R.adashift_fwd(xq, alpha, beta, d, z, bits, False, is_fc, bool(ht), bool(hr))
        if ht and hr:
            np.testing.assert_array_equal(y, g[k + "_y"], err_msg=k)   # all-integer path
        else:
            close(y, g[k + "_y"], rtol=1e-5, atol=1e-7)
        if not ht:
            ga, gb = R.adashift_bwd(xq, alpha, beta, d, z, bits, False, is_fc, bool(hr), g[tag + "_gy"])
            close(ga, g[k + "_galpha"], rtol=1e-4, atol=1e-6)
            if not hr:
                close(gb, g[k + "_gbeta"], rtol=1e-4, atol=1e-7)


@pytest.mark.parametrize("fname", CQ_FILES)
@pytest.mark.parametrize("tag", ["conv_b2", "conv_b4", "fc_b2", "fc_b4", "dw_b2", "dw_b4"])
def test_channelquant_lhs_and_adaround(golden, tag, fname):
    g = golden(fname)
    w, is_fc, d, z, bits = _cq_setup(g, tag)
    xq, alpha0 = R.init_v(w, d, z, bits, False, SHIFTS)
    np.testing.assert_array_equal(np.stack(xq), g[tag + "_lhs_xq"])
    close(alpha0, g[tag + "_lhs_alpha0"])
    alpha = g[tag + "_lhs_alpha"]
    close(R.shifted_x_quant(xq, alpha, is_fc, False), g[tag + "_lhs_t0_y"], atol=1e-7)
    np.testing.assert_array_equal(R.shifted_x_quant(xq, alpha, is_fc, True), g[tag + "_lhs_t1_y"])
    close(R.lhs_bwd(xq, alpha, is_fc, g[tag + "_gy"]), g[tag + "_lhs_t0_galpha"], rtol=1e-4, atol=1e-6)
    # adaround phase after update_delta (per (Co,Ci) delta)
    dsel = R.get_delta(d, alpha, SHIFTS, is_fc)
    np.testing.assert_array_equal(dsel, g[tag + "_ar_delta"])
    close(R.init_beta_from_delta(w, dsel), g[tag + "_ar_beta0"], atol=1e-5)
    beta = g[tag + "_ar_beta"]
    np.testing.assert_array_equal(R.adaround_fwd(w, beta, dsel, z, bits, False, True), g[tag + "_ar_r1_y"])
    close(R.adaround_fwd(w, beta, dsel, z, bits, False, False), g[tag + "_ar_r0_y"], atol=1e-7)
    close(R.adaround_bwd(w, beta, dsel, z, bits, False, g[tag + "_gy"]), g[tag + "_ar_r0_gbeta"],
          rtol=1e-4, atol=1e-7)
    np.testing.assert_array_equal(R.none_fwd(w, dsel, z, bits, False), g[tag + "_none_y"])


@pytest.mark.parametrize("fname", ["adaround", "adaround_specials"])
@pytest.mark.parametrize("name", ["conv", "fc"])
def test_adaround_quantizer(golden, name, fname):
    g = golden(fname)
    w = g[name + "_w"]
    shape = (-1, 1) if w.ndim == 2 else (-1, 1, 1, 1)
    d, z = g[name + "_delta"].reshape(shape), g[name + "_zp"].reshape(shape)
    close(R.init_beta_from_delta(w, d), g[name + "_alpha0"], atol=1e-5)
    a = g[name + "_alpha"]
    np.testing.assert_array_equal(R.adaround_fwd(w, a, d, z, 2, False, True), g[name + "_s0_y"])
    close(R.adaround_fwd(w, a, d, z, 2, False, False), g[name + "_s1_y"], atol=1e-7)
    close(R.adaround_bwd(w, a, d, z, 2, False, g[name + "_gy"]), g[name + "_s1_galpha"], rtol=1e-4, atol=1e-7)
    close(R.soft_round(a), g[name + "_h"])


# ------------------------------------------------------------------ K10
def test_inpscale(golden):
    g = golden("inpscale")
    for bits in (2, 4):
        w = g[f"b{bits}_w"]
        d = g[f"b{bits}_delta"].reshape(-1, 1, 1, 1)
        rz = g[f"b{bits}_rawzp"].reshape(-1, 1, 1, 1)
        for level in (1, 2, 8, 64):
            for thr in (1, 2):
                t = f"b{bits}_l{level}_t{thr}"
                inp = R.inpscale_search(w, d, rz, bits, level, float(thr))
                np.testing.assert_array_equal(inp, g[t + "_inp"], err_msg=t)
                np.testing.assert_array_equal(R.inpscale_fwd(w, inp, d, rz, bits), g[t + "_y"], err_msg=t)
    d, rz = g["fc_delta"].reshape(-1, 1), g["fc_rawzp"].reshape(-1, 1)
    inp = R.inpscale_search(g["fc_w"], d, rz, 2, 8, 2.0)
    np.testing.assert_array_equal(inp, g["fc_inp"])
    np.testing.assert_array_equal(R.inpscale_fwd(g["fc_w"], inp, d, rz, 2), g["fc_y"])


# ------------------------------------------------------------------ K11/K12 + schedules
def test_lp_loss(golden):
    g = golden("loss")
    for p in (1.0, 2.0, 2.4):
        for red in ("none", "all"):
            loss, grad = R.lp_loss(g["pred"], g["tgt"], p, red)
            close(loss, g[f"p{p}_{red}_loss"][0])
            close(grad, g[f"p{p}_{red}_grad"], rtol=1e-5, atol=1e-9)


def test_regularizers(golden):
    g = golden("loss")
    for b in (0.0, 20.0, 11.3, 2.0):
        l, ga = R.reg_shift(g["reg_alpha"], b, 0.1)
        close(l, g[f"regS_b{b}_loss"][0], rtol=1e-5)
        close(ga, g[f"regS_b{b}_grad"], rtol=1e-4, atol=1e-7)
        l, gb = R.reg_round(g["reg_beta"], b, 0.01)
        close(l, g[f"regR_b{b}_loss"][0], rtol=1e-5)
        close(gb, g[f"regR_b{b}_grad"], rtol=1e-4, atol=1e-7)
    l, ga = R.reg_entropy(g["reg_alpha"], 0.1)
    close(l, g["regE_loss"][0])
    close(ga, g["regE_grad"], rtol=1e-4, atol=1e-7)


def test_schedules(golden):
    g = golden("loss")
    for t in g["sched_t"]:
        t = int(t)
        assert R.linear_temp_decay(t, 100, guard_zero=True) == g["sched_fused"][t]
        assert R.linear_temp_decay(t, 75.0, guard_zero=True) == g["sched_fused_shift"][t]
        assert R.linear_temp_decay(t, 100) == g["sched_lin"][t]
        assert R.linear_temp_decay(t, 100) == g["sched_lsh"][t]


def test_recon_cpu_restatement_matches_reference_trajectory(golden):
    """oracle/recon_cpu.py (the CPU restatement bench.py times as the recon cpu_baseline)
    reproduces the reference's own 30-iteration block_recon_fused_shiftedScale run: the
    same batches, per-iteration reconstruction losses and final alphas."""
    import torch
    from oracle.recon_cpu import FusedBlockReconCPU
    g = golden("recon_fused")
    t = lambda a: torch.as_tensor(np.asarray(a))   # noqa: E731
    convs = {"conv1": (t(g["conv1_w"]), t(g["conv1_b"]), t(g["conv1_delta"]), t(g["conv1_zp"]), 2, 1),
             "conv2": (t(g["conv2_w"]), t(g["conv2_b"]), t(g["conv2_delta"]), t(g["conv2_zp"]), 1, 1),
             "downsample": (t(g["downsample_w"]), t(g["downsample_b"]), t(g["downsample_delta"]),
                            t(g["downsample_zp"]), 2, 0)}
    iters = int(g["iters"][0])
    torch.manual_seed(1005)
    rc = FusedBlockReconCPU(convs, [31 / 32, 33 / 32, 1.0], 2, t(g["cached_inp"]), t(g["cached_out"]),
                            iters)
    rec = [rc.step() for _ in range(iters)]
    np.testing.assert_allclose(rec, g["rec_loss"][:iters], rtol=1e-5)
    for n in ("conv1", "conv2", "downsample"):
        # rows whose shift candidates are all equal have a zero analytic gradient: Adam turns
        # summation-order noise into +-lr steps there (in the reference too), bounded below
        fl = torch.stack(rc.convs[n].floors).numpy()
        degenerate = np.all(fl == fl[:1], axis=(0, 1, 3, 4))
        da = np.abs(rc.convs[n].alpha.detach().numpy() - g[n + "_alpha"])
        assert da[~degenerate].max() <= 1e-5, (n, da[~degenerate].max())
        assert da.max() <= iters * 2e-3, n
