"""Reconstruction loops on the GPU against the reference's own trajectories
(tests/golden/recon_*.npz, produced by make_golden.py from the reference on CPU).

The loops are seeded exactly like the reference (torch.manual_seed(1005), CPU randperm),
so every batch drawn is identical (checked); per-iteration losses and the learned
parameters then agree up to conv/summation rounding (MIOpen vs mkldnn), which is what
the tolerances below bound.  Hard decisions that ride on near-ties of two shift
probabilities may flip: their count is bounded explicitly.
"""
import numpy as np
import pytest
import torch
import torch.nn as nn

from conftest import assert_hard_flips_bounded, assert_shift_flips_bounded, assert_walk_bounded

pytestmark = pytest.mark.gpu
SHIFTS = [31 / 32, 33 / 32, 1.0]


@pytest.fixture(scope="module")
def Q():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from shiftedscalequantization_amd import quant
    return quant


def dev(a):
    return torch.as_tensor(np.asarray(a)).cuda()


def parity_report(test, **stats):
    """Print the reached parity and append it to $SSQ_PARITY_LOG (jsonl) when set."""
    import json
    import os
    rec = {"test": test, **{k: float(v) for k, v in stats.items()}}
    print("PARITY", json.dumps(rec))
    path = os.environ.get("SSQ_PARITY_LOG")
    if path:
        with open(path, "a") as f:
            f.write(json.dumps(rec) + "\n")


@pytest.fixture(params=["never", "always"])
def wgrad(request):
    """Conv weight gradients from MIOpen ('never') or from K17 ssq_conv_wgrad ('always')."""
    from shiftedscalequantization_amd import kernels
    old, kernels.WGRAD_POLICY = kernels.WGRAD_POLICY, request.param
    yield request.param
    kernels.WGRAD_POLICY = old


@pytest.fixture
def det_convs():
    """MIOpen's deterministic conv solvers (the reference's seed_all setting): in the default
    mode its stride-2 weight gradients may accumulate with atomics, so two runs of the same
    loop can differ in the last bits; tests that compare two loop runs bit for bit use this."""
    cudnn = torch.backends.cudnn
    old = cudnn.deterministic
    cudnn.deterministic = True
    yield
    cudnn.deterministic = old


def tiny_net():
    """Same topology as make_golden._tiny_net (weights are loaded from the fixture)."""
    from shiftedscalequantization_amd import nets
    ds = nn.Sequential(nn.Conv2d(16, 32, 1, stride=2, bias=False), nn.BatchNorm2d(32))
    return nn.Sequential(nn.Conv2d(3, 16, 3, padding=1, bias=False), nn.BatchNorm2d(16), nn.ReLU(),
                         nets.BasicBlock(16, 32, stride=2, downsample=ds),
                         nn.AdaptiveAvgPool2d(1), nn.Flatten(), nn.Linear(32, 10)).eval()


def build_qnn(Q, g, bits_w=2, bits_a=4, net=None):
    wq = {"n_bits": bits_w, "channel_wise": True, "scale_method": "max"}
    aq = {"n_bits": bits_a, "channel_wise": False, "scale_method": "mse", "leaf_param": True}
    qnn = Q.QuantModel(tiny_net() if net is None else net, wq, aq).cuda().eval()
    qnn.set_first_last_layer_to_8bit()
    qms = [m for m in qnn.modules() if isinstance(m, Q.QuantModule)]
    for k, m in enumerate(qms):
        if f"qm{k}_w" not in g:
            continue
        w, b = dev(g[f"qm{k}_w"]), dev(g[f"qm{k}_b"])
        m.org_weight = w.clone()
        m.weight.data = w.clone()
        m.org_bias = b.clone()
        m.bias.data = b.clone()
        shape = (-1,) + (1,) * (w.dim() - 1)
        m.weight_quantizer.delta = nn.Parameter(dev(g[f"qm{k}_delta"]).view(shape))
        m.weight_quantizer.zero_point = nn.Parameter(dev(g[f"qm{k}_zp"]).view(shape))
        m.weight_quantizer.inited = True
    return qnn


def load_block(Q, g, block):
    for n in ("conv1", "conv2", "downsample"):
        m = getattr(block, n)
        w, b = dev(g[n + "_w"]), dev(g[n + "_b"])
        m.org_weight, m.org_bias = w.clone(), b.clone()
        m.weight.data = w.clone()
        m.bias = nn.Parameter(b.clone())
        uaq = Q.UniformAffineQuantizer(n_bits=2, channel_wise=True, ch=w.shape).cuda()
        uaq.delta = nn.Parameter(dev(g[n + "_delta"]).view(-1, 1, 1, 1))
        uaq.zero_point = nn.Parameter(dev(g[n + "_zp"]).view(-1, 1, 1, 1))
        uaq.inited = True
        m.weight_quantizer = Q.ChannelQuant(1.0, uaq=uaq, weight_tensor=m.org_weight, shiftTarget=SHIFTS,
                                            name="." + n)
        m.use_weight_quant = True


@pytest.mark.parametrize("bias_cal", [False, True])
@pytest.mark.parametrize("graph", [False, True])
def test_block_recon_fused_matches_reference(Q, golden, graph, wgrad, bias_cal):
    """bias_cal=True: against the reference run with --bias_cal's commented opt_params
    lines realised (recon_fused_biascal.npz, make_golden._BiasCalAdam): gamma^z / phi^z
    follow the reference's trajectory too."""
    g = golden("recon_fused_biascal" if bias_cal else "recon_fused")
    qnn = build_qnn(Q, {})
    block = qnn.model[3]
    load_block(Q, g, block)
    block.cached_inp_features = [dev(g["cached_inp"])]
    block.cached_out_features = [dev(g["cached_out"])]
    iters = int(g["iters"][0])

    import importlib
    LRF = importlib.import_module("shiftedscalequantization_amd.quant.layer_recon_fused_shiftedScale")
    seen_perms, seen_rec = [], []
    orig_draw = LRF.BatchFeeder.draw
    orig_keep = LRF.FusedScaleLossFunction.bookkeep

    def draw(self):
        p = orig_draw(self)
        seen_perms.append(p.clone())
        return p

    def bookkeep(self, rec):
        seen_rec.append(float(rec.item()))     # read now: a graph replay overwrites it
        return orig_keep(self, rec)

    LRF.BatchFeeder.draw, LRF.FusedScaleLossFunction.bookkeep = draw, bookkeep
    try:
        torch.manual_seed(1005)
        res = LRF.block_recon_fused_shiftedScale(block, iters, (0.01, 0.1), qnn, None, verbose=False,
                                                 graph=graph, bias_cal=bias_cal)
    finally:
        LRF.BatchFeeder.draw, LRF.FusedScaleLossFunction.bookkeep = orig_draw, orig_keep
    # identical batches (same CPU RNG stream as the reference)
    np.testing.assert_array_equal(np.stack([p.numpy() for p in seen_perms]), g["perms"])
    rec = np.array(seen_rec)
    stats = {"rec_rel_err": np.max(np.abs(rec - g["rec_loss"][:iters]) / np.abs(g["rec_loss"][:iters])),
             "final_rel_err": np.max(np.abs(np.array(res) - g["final_losses"]) / np.abs(g["final_losses"]))}
    # observed (r2, MI355X): rec / final rel err <= 8e-7, alpha dev <= 5e-7, 0 hard flips
    np.testing.assert_allclose(rec, g["rec_loss"][:iters], rtol=1e-5)
    np.testing.assert_allclose(res, g["final_losses"], rtol=1e-5)
    for n in ("conv1", "conv2", "downsample"):
        q = getattr(block, n).weight_quantizer
        # Input channels whose shift candidates are all identical (floor(W/(d*s_i)) equal
        # for every shift, common in 1x1 convs) have an analytically ZERO alpha gradient;
        # Adam turns the rounding noise left there into full +-lr steps in both the
        # reference and here, so those rows are a random walk of a few lr-steps.  Every
        # other row must follow the reference trajectory.
        from oracle import ssq_ref as R
        w = g[n + "_w"]
        fl = np.stack(R.shift_floors(w, g[n + "_delta"].reshape(-1, 1, 1, 1), SHIFTS))
        degenerate = np.all(fl == fl[:1], axis=(0, 1, 3, 4))          # per input channel
        da = np.abs(q.alpha.detach().cpu().numpy() - g[n + "_alpha"])
        stats[n + "_alpha_dev"] = da[~degenerate].max()
        stats[n + "_alpha_dev_degenerate"] = da[degenerate].max(initial=0.0)
        stats[n + "_alpha_walkers"] = assert_walk_bounded(da[~degenerate], 1e-5, 30 * 2e-3,
                                                          what=n)
        assert da[degenerate].max(initial=0.0) <= 30 * 1e-3 * 2, n      # <= iters * 2 lr
        np.testing.assert_allclose(q.beta.detach().cpu().numpy(), g[n + "_beta0"], rtol=1e-5, atol=1e-5)
        with torch.no_grad():
            what = q(getattr(block, n).weight).cpu().numpy()
        stats[n + "_hard_flips"] = assert_shift_flips_bounded(
            what, g[n + "_what_hard"], q.alpha.detach().cpu().numpy(), g[n + "_alpha"],
            iters * 2e-3, n)
        if bias_cal:
            m = getattr(block, n)
            for key, t in (("gamma", m.alpha_out), ("phi", m.beta_out)):
                d_ = np.abs(t.detach().cpu().numpy().reshape(-1) - g[f"{n}_{key}"].reshape(-1))
                stats[f"{n}_{key}_dev"] = d_.max()
                stats[f"{n}_{key}_walkers"] = assert_walk_bounded(d_, 1e-5, iters * 2e-3, frac=0.05,
                                                                  what=n + key)
    parity_report(f"a18_block_recon_fused[graph={graph},wgrad={wgrad},bias_cal={bias_cal}]", **stats)


def test_layer_recon_shiftedScale_matches_reference(Q, golden):
    g = golden("recon_layer_shift")
    qnn = build_qnn(Q, {}, bits_w=4, bits_a=8)
    m = qnn.model[3].conv1
    w, b = dev(g["w"]), dev(g["b"])
    m.org_weight, m.org_bias = w.clone(), b.clone()
    m.weight.data = w.clone()
    m.bias = nn.Parameter(b.clone())
    uaq = Q.UniformAffineQuantizer(n_bits=4, channel_wise=True, ch=w.shape).cuda()
    uaq.delta = nn.Parameter(dev(g["delta"]).view(-1, 1, 1, 1))
    uaq.zero_point = nn.Parameter(dev(g["zp"]).view(-1, 1, 1, 1))
    uaq.inited = True
    m.weight_quantizer = Q.ChannelQuant(1.0, uaq=uaq, weight_tensor=w, shiftTarget=SHIFTS, name="c1")
    m.use_weight_quant = True
    m.cached_inp_features = [dev(g["cached_inp"])]
    m.cached_out_features = [dev(g["cached_out"])]
    iters = int(g["iters"][0])
    torch.manual_seed(1005)
    l1 = Q.layer_recon_shiftedScale(m, iters, 0.1, qnn, None, verbose=False)
    stats = {"shift_final_rel_err": np.max(np.abs(np.array(l1) - g["shift_final"]) / np.abs(g["shift_final"])),
             "shift_alpha_dev": np.abs(m.weight_quantizer.alpha.detach().cpu().numpy() - g["shift_alpha"]).max()}
    # observed (r2): final rel err <= 5e-7, alpha dev 4.4e-7, 0 delta flips, beta dev 2.4e-4
    np.testing.assert_allclose(l1, g["shift_final"], rtol=1e-5)
    assert_walk_bounded(np.abs(m.weight_quantizer.alpha.detach().cpu().numpy() - g["shift_alpha"]),
                        1e-5, iters * 2e-3, what="shift alpha")
    m.weight_quantizer.hard_targets = False
    l2 = Q.layer_recon_shiftedScale(m, iters, 0.01, qnn, None, adaround=True, verbose=False)
    np.testing.assert_allclose(l2, g["ar_final"], rtol=1e-5)
    d = m.weight_quantizer.delta.detach().cpu().numpy()
    stats["ar_final_rel_err"] = np.max(np.abs(np.array(l2) - g["ar_final"]) / np.abs(g["ar_final"]))
    stats["ar_delta_flips"] = np.sum(d != g["ar_delta"])
    stats["ar_beta_dev"] = np.abs(m.weight_quantizer.beta.detach().cpu().numpy() - g["ar_beta"]).max()
    stats["ar_beta_walkers"] = np.mean(np.abs(m.weight_quantizer.beta.detach().cpu().numpy() - g["ar_beta"]) > 2e-4)
    parity_report("a20_layer_recon_shiftedScale", **stats)
    assert np.mean(d != g["ar_delta"]) <= 0.005
    # beta entries whose rounding-loss gradient nearly cancels are walked by Adam in +-lr
    # steps, and which entries do depends on the fp32 summation order of the box's conv
    # weight-gradient solver (observed r2: 11 of 4608 off by up to 1.6e-3 on one box, 154
    # on another, none above 2.4e-4 on a third).  Bounded by what Adam can do: no entry
    # moves more than its step budget, most stay tight, and the hard rounding decision
    # (h(beta) >= 0.5 <=> beta >= 0) agrees wherever the reference's beta is further from 0
    # than that budget.
    budget = iters * 2 * 1e-3
    bq = m.weight_quantizer.beta.detach().cpu().numpy()
    db = np.abs(bq - g["ar_beta"])
    assert np.mean(db > 2e-4) <= 0.05, np.mean(db > 2e-4)
    assert db.max() <= budget
    decided = np.abs(g["ar_beta"]) > budget
    assert np.all((bq >= 0)[decided] == (g["ar_beta"] >= 0)[decided])


@pytest.mark.parametrize("graph", [False, True])
@pytest.mark.parametrize("fixture", ["recon_brecq", "recon_brecq_long", "recon_brecq_affine"])
def test_brecq_block_reconstruction_matches_reference(Q, golden, graph, wgrad, fixture):
    """a22 BRECQ block_reconstruction, AdaRound weight phase then the act-delta phase, against
    the reference's trajectory: 10 iterations, 400 (recon_brecq_long: the b schedule's end,
    the act phase's cosine LR decayed to zero), and 50 with non-identity gamma^z / phi^z
    (recon_brecq_affine: the --bias_cal flow's act phase -- general K13 epilogue, fused tail
    at p = 2.4, deferred delta finalize with the riding Adam step, pinned weights)."""
    g = golden(fixture)
    qnn = build_qnn(Q, g)
    block = qnn.model[3]
    if "conv1_gamma" in g:
        for n in ("conv1", "conv2", "downsample"):
            m = getattr(block, n)
            with torch.no_grad():
                m.alpha_out.copy_(dev(g[n + "_gamma"]))
                m.beta_out.copy_(dev(g[n + "_phi"]))
    cali = dev(g["cali"])
    import importlib
    BR = importlib.import_module("shiftedscalequantization_amd.quant.block_recon")
    seen = []
    orig_rec, orig_init = BR.LossFunction.record, BR.LossFunction.__init__

    def spy(self, rec, rnd, b):
        r = orig_rec(self, rec, rnd, b)
        seen.append(float(r))          # read now: a graph replay overwrites it
        return r

    def init(self, *a, **k):
        orig_init(self, *a, **k)
        self.track_values = True       # the round value every iteration, for the comparison

    BR.LossFunction.record, BR.LossFunction.__init__ = spy, init
    orig_fast = BR._fast_loop
    BR._fast_loop = lambda *a: orig_fast(*(a[:-1] + (a[-1] and graph,)))
    try:
        torch.manual_seed(1005)
        Q.block_reconstruction(qnn, block, cali, batch_size=8, iters=len(g["w_total_loss"]),
                               weight=0.01, asym=True, b_range=(20, 2), warmup=0.2,
                               act_quant=False, opt_mode="mse")
        stats = {"w_total_rel_err": np.max(np.abs(np.array(seen) - g["w_total_loss"]) /
                                           np.abs(g["w_total_loss"]))}
        # observed (r2): total rel err <= 6.2e-7, V dev <= 4.7e-7, 0 flips, act delta 2e-7
        np.testing.assert_allclose(seen, g["w_total_loss"], rtol=1e-5)
        for n in ("conv1", "conv2", "downsample"):
            q = getattr(block, n).weight_quantizer
            dv = np.abs(q.alpha.detach().cpu().numpy() - g[n + "_alpha"])
            stats[n + "_V_dev"] = dv.max()
            # 400 iterations (recon_brecq_long) under MIOpen's default stride-2 weight gradients,
            # which may accumulate with atomics: V entries with a near-zero gradient walk by
            # a few 1e-5 (observed r4: up to 8e-5 on 1.2 % of conv1's entries in one run, none
            # in another) -- tight at 1e-4 there, 1e-5 at 10 / 50 iterations
            tight = 1e-4 if fixture == "recon_brecq_long" else 1e-5
            stats[n + "_V_walkers"] = assert_walk_bounded(dv, tight, len(seen) * 2e-3, what=n)
            with torch.no_grad():
                what = q(getattr(block, n).weight).cpu().numpy()
            stats[n + "_hard_flips"] = assert_hard_flips_bounded(
                what, g[n + "_what_hard"], q.alpha.detach().cpu().numpy(), g[n + "_alpha"],
                len(seen) * 2e-3, n)
        # act phase
        qnn.set_quant_state(True, True)
        with torch.no_grad():
            qnn(cali[:8])
        qnn.disable_network_output_quantization()
        aqs = [block.act_quantizer] + [m.act_quantizer for m in (block.conv1, block.conv2, block.downsample)
                                       if m.act_quantizer.delta is not None]
        np.testing.assert_allclose([float(q.delta) for q in aqs], g["a_delta0"], rtol=1e-6)
        stats["a_delta0_rel_err"] = np.max(np.abs(np.array([float(q.delta) for q in aqs]) - g["a_delta0"]) /
                                           g["a_delta0"])
        if fixture == "recon_brecq_long":
            # the act phase from the reference's own start state: its weight phase's V (the
            # hard W^ then bit-identical, flips or not) and its act-delta init, so the act
            # comparison below measures the act phase only
            with torch.no_grad():
                for n in ("conv1", "conv2", "downsample"):
                    getattr(block, n).weight_quantizer.alpha.copy_(dev(g[n + "_alpha"]))
                for q, d0 in zip(aqs, g["a_delta0"]):
                    q.delta.fill_(float(d0))
        seen.clear()
        torch.manual_seed(1005)
        Q.block_reconstruction(qnn, block, cali, batch_size=8, iters=len(g["a_total_loss"]),
                               act_quant=True, opt_mode="mse", lr=4e-4, p=2.4)
        stats["a_total_rel_err"] = np.max(np.abs(np.array(seen) - g["a_total_loss"]) / np.abs(g["a_total_loss"]))
        stats["a_delta_rel_err"] = np.max(np.abs(np.array([float(q.delta) for q in aqs]) - g["a_delta"]) /
                                          np.abs(g["a_delta"]))
        a_rel = np.abs(np.array(seen) - g["a_total_loss"]) / np.abs(g["a_total_loss"])
        if fixture == "recon_brecq_long":
            # The act phase is chaotic over hundreds of steps: a delta one rounding away from
            # another flips some activations' rounding, and the trajectory wanders off.  The
            # reference itself, its act deltas nudged by ONE fp32 ulp, drifts from its own
            # recorded trajectory by as much as this run does (tests/golden/
            # brecq_sensitivity.py -> profiles/r4_brecq_act_sensitivity.json: losses max 3.9e-3 /
            # median 1.7e-4, 100-iteration means <= 1.5e-4, final deltas 7.5e-4; this run,
            # r4: 3.7e-3 / 1.7e-4, <= 1.8e-4, 7.9e-4).  So: the first 20 iterations tight,
            # then the reference's own one-ulp spread.
            win = [abs(np.mean(seen[i:i + 100]) - np.mean(g["a_total_loss"][i:i + 100])) /
                   np.mean(g["a_total_loss"][i:i + 100]) for i in range(0, len(seen), 100)]
            stats["a_window_mean_rel_err"] = max(win)
            stats["a_median_rel_err"] = float(np.median(a_rel))
            l64 = g["a_total_loss64"]
            k = len(l64)
            stats["a_first20_rel_err"] = a_rel[:k].max()
            stats["a_first20_argmax"] = int(a_rel[:k].argmax())
            stats["a_first20_ours_vs_f64"] = np.max(np.abs(np.array(seen[:k]) - l64) / l64)
            stats["a_first20_ref_vs_f64"] = np.max(np.abs(g["a_total_loss"][:k] - l64) / l64)
        parity_report(f"a22_brecq_basic[{fixture},graph={graph},wgrad={wgrad}]", **stats)
        if fixture == "recon_brecq_long":
            # first 20 act iterations, from the reference's start state (above): the
            # reference is within 1.2e-7 of float64 there (a_total_loss64, no activation
            # rounding decided differently), so 1e-5 leaves room only for the convs'
            # summation order.  r5 held 5e-5 after one box type reached 2.3e-5 while the act
            # phase started from our own delta init (rtol 1e-6 of the reference's) -- not from
            # the weight phase, whose hard W^ had no flip: 0 of every conv's decisions
            assert a_rel[:20].max() <= 1e-5, a_rel[:20].max()
            assert np.median(a_rel) <= 1e-3 and a_rel.max() <= 1e-2, (np.median(a_rel), a_rel.max())
            assert max(win) <= 1e-3, win
            np.testing.assert_allclose([float(q.delta) for q in aqs], g["a_delta"], rtol=2e-3)
        elif fixture == "recon_brecq_affine":
            # 50 act iterations: a loss value can carry one activation that rounds the other
            # way (a delta one rounding away; MIOpen's default stride-2 weight gradients make
            # the weight phase's last bits vary run to run).  Observed r4: in one run of four
            # one iteration at 1.8e-4, deltas 3.4e-7 -- at most 2 such iterations, <= 1e-3
            odd = a_rel > 1e-5
            stats["a_odd_iterations"] = int(odd.sum())
            assert odd.sum() <= 2 and a_rel.max() <= 1e-3, (int(odd.sum()), a_rel.max())
            np.testing.assert_allclose([float(q.delta) for q in aqs], g["a_delta"], rtol=5e-6)
        else:
            np.testing.assert_allclose(seen, g["a_total_loss"], rtol=1e-5)
            np.testing.assert_allclose([float(q.delta) for q in aqs], g["a_delta"], rtol=5e-6)
    finally:
        BR.LossFunction.record, BR.LossFunction.__init__ = orig_rec, orig_init
        BR._fast_loop = orig_fast


@pytest.mark.parametrize("rows", [False, True])
@pytest.mark.parametrize("graph", [False, True])
@pytest.mark.parametrize("affine", [False, True])
def test_brecq_loop_knobs_bit_identical(Q, golden, graph, affine, rows, det_convs):
    """block_recon._fast_loop's launch savings -- deferred finalizes, the fused tail (p = 2
    weight phase, p = 2.4 act phase), the act phase's pinned weights and its precomputed
    block-input convs (conv1, the downsample: gathered rows instead of the conv) -- against the plain
    loop: AdaRound V, the act deltas and the Adam moments bit-identical after each phase,
    per-iteration losses equal to the last float ulps (row-wise vs block-wise loss partials).
    affine: gamma^z / phi^z live (the --bias_cal flow's act phase: the general K13 epilogue,
    whose delta gradient the fused tail and the deferred finalize produce).  rows: the cached
    convs' rows read in place by the epilogue kernels (ROWS_IN_PLACE: no gather launch at all
    in the act phase, no row view gathered behind the loop's back) instead of gathered."""
    import importlib
    BR = importlib.import_module("shiftedscalequantization_amd.quant.block_recon")
    E = importlib.import_module("shiftedscalequantization_amd.quant._engine")
    g = golden("recon_brecq")
    views, fallbacks = [], []
    cali = dev(g["cali"])
    runs, used = [], []
    for on in (False, True):
        qnn = build_qnn(Q, g)
        block = qnn.model[3]
        if affine:
            gen = torch.Generator().manual_seed(7)
            for n in ("conv1", "conv2", "downsample"):
                m = getattr(block, n)
                with torch.no_grad():
                    m.alpha_out.copy_(1 + 0.05 * torch.randn(m.alpha_out.shape, generator=gen))
                    m.beta_out.copy_(0.02 * torch.randn(m.beta_out.shape, generator=gen))
        seen, opts, tails, pins, cconvs, stashed = [], [], [], [], [], []
        orig_rec, orig_init = BR.LossFunction.record, E.SsqAdam.__init__
        orig_tail, orig_pin, orig_cc = BR.K.epilogue_loss_bwd, BR.pinned_weights, BR.cached_convs
        orig_stash = BR.stash_adaround

        def spy(self, rec, rnd, b):
            r = orig_rec(self, rec, rnd, b)
            seen.append(float(r))
            return r

        def init(self, *a, **k):
            orig_init(self, *a, **k)
            opts.append(self)

        def tail(*a, **k):
            tails.append(1)
            return orig_tail(*a, **k)

        def pin(mods):
            pins.append(1)
            return orig_pin(mods)

        def cc(mods, *a, **k):
            cconvs.append(len(mods))
            return orig_cc(mods, *a, **k)

        orig_gather, pairs = BR.K.gather_rows2, []

        def gather(src0, idx, src1=None, **k):
            pairs.append(src1 is not None)
            return orig_gather(src0, idx, src1, **k)

        def stash(mods):
            orig_stash(mods)
            stashed.append(sum(getattr(m.weight_quantizer, "_stash", None) is not None for m in mods))

        knobs = {k: getattr(BR, k) for k in ("DEFER_FINALIZE", "FUSE_TAIL", "PIN_WEIGHTS",
                                             "CACHE_CONVS", "STASH_ADAROUND", "GATHER_ONCE",
                                             "ROWS_IN_PLACE")}
        BR.LossFunction.record, E.SsqAdam.__init__, BR.K.epilogue_loss_bwd = spy, init, tail
        BR.pinned_weights, BR.cached_convs, BR.stash_adaround = pin, cc, stash
        orig_fast = BR._fast_loop
        BR._fast_loop = lambda *a: orig_fast(*(a[:-1] + (a[-1] and graph,)))
        orig_view, orig_mat = BR.K.rows_view, BR.K.A.materialize_rows

        def view(*a):
            views.append(1)
            return orig_view(*a)

        def mat(t):
            if t.data_ptr() in BR.K.A.ROW_VIEWS:
                fallbacks.append(1)
            return orig_mat(t)

        BR.K.rows_view, BR.K.A.materialize_rows = view, mat
        for k in knobs:
            setattr(BR, k, on and (rows or k != "ROWS_IN_PLACE"))
        out = {}
        try:
            torch.manual_seed(1005)
            Q.block_reconstruction(qnn, block, cali, batch_size=8, iters=12, weight=0.01,
                                   asym=True, b_range=(20, 2), warmup=0.2, act_quant=False,
                                   opt_mode="mse")
            out["w_rec"] = np.array(seen)
            for n in ("conv1", "conv2", "downsample"):
                out[n + "_V"] = getattr(block, n).weight_quantizer.alpha.detach().cpu().numpy()
            qnn.set_quant_state(True, True)
            with torch.no_grad():
                qnn(cali[:8])
            qnn.disable_network_output_quantization()
            seen.clear()
            torch.manual_seed(1005)
            BR.K.gather_rows2 = gather
            Q.block_reconstruction(qnn, block, cali, batch_size=8, iters=12, act_quant=True,
                                   opt_mode="mse", lr=4e-4, p=2.4)
            BR.K.gather_rows2 = orig_gather
            out["a_rec"] = np.array(seen)
            aqs = [block.act_quantizer] + [m.act_quantizer for m in (block.conv1, block.conv2,
                                                                      block.downsample)
                                           if m.act_quantizer.delta is not None]
            out["a_delta"] = np.array([float(q.delta) for q in aqs])
            for k, o in enumerate(opts):
                for j, p_ in enumerate(o.params):
                    out[f"opt{k}_m{j}"] = o.state[p_]["exp_avg"].cpu().numpy()
                    out[f"opt{k}_v{j}"] = o.state[p_]["exp_avg_sq"].cpu().numpy()
        finally:
            BR.LossFunction.record, E.SsqAdam.__init__, BR.K.epilogue_loss_bwd = orig_rec, orig_init, orig_tail
            BR.pinned_weights, BR._fast_loop, BR.cached_convs = orig_pin, orig_fast, orig_cc
            BR.stash_adaround, BR.K.gather_rows2 = orig_stash, orig_gather
            BR.K.rows_view, BR.K.A.materialize_rows = orig_view, orig_mat
            for k, v in knobs.items():
                setattr(BR, k, v)
        runs.append(out)
        used.append((len(tails), len(pins), cconvs, sorted(set(stashed)), sorted(set(pairs))))
    # the act phase caches conv1 and the downsample (both read the block input) and gathers
    # both their rows in one launch per iteration (the plain loop: the batch input only) --
    # or, rows, gathers nothing (the input is not read; the epilogues read the cached rows in
    # place); the weight phase computes the block's three AdaRound weights in one launch
    assert used[0] == (0, 0, [], [], [False]) and used[1][0] > 0 and used[1][1] == 1 \
        and used[1][2] == [2] and used[1][3] == [3] and used[1][4] == ([] if rows else [True]), used
    assert (len(views) > 0) == rows and not fallbacks, (len(views), len(fallbacks))
    assert runs[0].keys() == runs[1].keys()
    for k in runs[0]:
        if k.endswith("_rec"):
            np.testing.assert_allclose(runs[1][k], runs[0][k], rtol=1e-6, err_msg=k)
        else:
            np.testing.assert_array_equal(runs[1][k], runs[0][k], err_msg=k)


@pytest.mark.parametrize("graph", [False, True])
def test_brecq_layer_reconstruction_matches_reference(Q, golden, graph):
    """a22, BRECQ's per-layer path (layer_recon.py:10-104 + its LossFunction :107-170) as
    recon_model calls it for QuantModules: the block's conv1 then the fc (whose captured
    input carries conv1's finished hard rounding), AdaRound weight phase, then the act-delta
    phase (the fc's act quantizer is the disabled network output: loss only, delta
    untouched), against recon_layer_brecq.npz."""
    g = golden("recon_layer_brecq")
    qnn = build_qnn(Q, g)
    cali = dev(g["cali"])
    iters = int(g["iters"][0])
    layers = [("conv", qnn.model[3].conv1), ("fc", qnn.model[6])]
    assert layers[1][1].weight.dim() == 2
    import importlib
    BR = importlib.import_module("shiftedscalequantization_amd.quant.block_recon")
    seen = []
    orig_rec, orig_init, orig_fast = BR.LossFunction.record, BR.LossFunction.__init__, BR._fast_loop

    def spy(self, rec, rnd, b):
        r = orig_rec(self, rec, rnd, b)
        seen.append(float(r))
        return r

    def init(self, *a, **k):
        orig_init(self, *a, **k)
        self.track_values = True

    BR.LossFunction.record, BR.LossFunction.__init__ = spy, init
    BR._fast_loop = lambda *a: orig_fast(*(a[:-1] + (a[-1] and graph,)))
    stats = {}
    try:
        for tag, layer in layers:
            seen.clear()
            torch.manual_seed(1005)
            Q.layer_reconstruction(qnn, layer, cali, batch_size=8, iters=iters, weight=0.01, asym=True,
                                   b_range=(20, 2), warmup=0.2, act_quant=False, opt_mode="mse")
            stats[tag + "_w_total_rel_err"] = np.max(np.abs(np.array(seen) - g[tag + "_w_total_loss"]) /
                                                     np.abs(g[tag + "_w_total_loss"]))
            np.testing.assert_allclose(seen, g[tag + "_w_total_loss"], rtol=1e-5)
            q = layer.weight_quantizer
            dv = np.abs(q.alpha.detach().cpu().numpy() - g[tag + "_alpha"])
            stats[tag + "_V_dev"] = dv.max()
            stats[tag + "_V_walkers"] = assert_walk_bounded(dv, 1e-5, iters * 2e-3, what=tag)
            with torch.no_grad():
                what = q(layer.weight).cpu().numpy()
            stats[tag + "_hard_flips"] = assert_hard_flips_bounded(
                what, g[tag + "_what_hard"], q.alpha.detach().cpu().numpy(), g[tag + "_alpha"],
                iters * 2e-3, tag)
        qnn.set_quant_state(True, True)
        with torch.no_grad():
            qnn(cali[:8])
        qnn.disable_network_output_quantization()
        for tag, layer in layers:
            aq = layer.act_quantizer
            np.testing.assert_allclose([float(aq.delta)], g[tag + "_a_delta0"], rtol=1e-6)
            assert int(not aq.disable_act_quant and not layer.disable_act_quant) == int(g[tag + "_a_on"][0])
            seen.clear()
            torch.manual_seed(1005)
            Q.layer_reconstruction(qnn, layer, cali, batch_size=8, iters=iters, act_quant=True,
                                   opt_mode="mse", lr=4e-4, p=2.4)
            stats[tag + "_a_total_rel_err"] = np.max(np.abs(np.array(seen) - g[tag + "_a_total_loss"]) /
                                                     np.abs(g[tag + "_a_total_loss"]))
            stats[tag + "_a_delta_rel_err"] = abs(float(aq.delta) - g[tag + "_a_delta"][0]) / g[tag + "_a_delta"][0]
            # the fc's act quantizer is the disabled network output: its "loss" is the fp32
            # noise between two evaluations of the same quantized layer (~7e-7, a sum of
            # squares of near-cancelling differences) -- agreeing to ~2e-5 relative is what
            # fp32 convs / GEMMs in another summation order give there
            rtol = 1e-5 if int(g[tag + "_a_on"][0]) else 1e-4
            np.testing.assert_allclose(seen, g[tag + "_a_total_loss"], rtol=rtol)
            np.testing.assert_allclose([float(aq.delta)], g[tag + "_a_delta"], rtol=5e-6)
        with torch.no_grad():
            logits = qnn(cali).cpu().numpy()
        stats["logits_rel_err"] = np.abs(logits - g["logits"]).max() / np.abs(g["logits"]).max()
        assert stats["logits_rel_err"] <= 1e-4
    finally:
        BR.LossFunction.record, BR.LossFunction.__init__, BR._fast_loop = orig_rec, orig_init, orig_fast
        parity_report(f"a22_layer_reconstruction[graph={graph}]", **stats)


@pytest.mark.parametrize("rows", [False, True])
@pytest.mark.parametrize("affine", [False, True])
def test_brecq_act_identity_block_gathers_input_with_conv(Q, affine, rows, det_convs):
    """BRECQ's act phase on a block with an identity residual (no downsample, e.g. ResNet-18
    layer1.1): the block input is still read (the residual), so each iteration gathers it
    together with the cached conv1 rows in ONE ssq_gather_rows2 launch (GATHER_ONCE) -- or,
    rows (ROWS_IN_PLACE), gathers nothing: conv1's epilogue reads the cached conv1 rows and
    the fused tail the residual's cached input rows in place; act deltas and Adam moments
    bit-identical to the plain loop (every knob off), losses to the last ulps."""
    import importlib
    from shiftedscalequantization_amd import nets
    BR = importlib.import_module("shiftedscalequantization_amd.quant.block_recon")
    E = importlib.import_module("shiftedscalequantization_amd.quant._engine")
    knobs = ("DEFER_FINALIZE", "FUSE_TAIL", "PIN_WEIGHTS", "CACHE_CONVS", "STASH_ADAROUND",
             "GATHER_ONCE", "ROWS_IN_PLACE")
    gen = torch.Generator().manual_seed(21)
    fallbacks = []
    cali = torch.randn(32, 3, 12, 12, generator=gen).cuda()
    runs, pairs = [], []
    for on in (False, True):
        torch.manual_seed(5)
        net = nn.Sequential(nn.Conv2d(3, 16, 3, padding=1, bias=False), nn.BatchNorm2d(16),
                            nn.ReLU(), nets.BasicBlock(16, 16), nn.AdaptiveAvgPool2d(1),
                            nn.Flatten(), nn.Linear(16, 10)).eval()
        qnn = Q.QuantModel(net, {"n_bits": 2, "channel_wise": True, "scale_method": "max"},
                           {"n_bits": 4, "channel_wise": False, "scale_method": "mse",
                            "leaf_param": True}).cuda().eval()
        qnn.set_first_last_layer_to_8bit()
        block = qnn.model[3]
        if affine:
            g2 = torch.Generator().manual_seed(7)
            for n in ("conv1", "conv2"):
                m = getattr(block, n)
                with torch.no_grad():
                    m.alpha_out.copy_(1 + 0.05 * torch.randn(m.alpha_out.shape, generator=g2))
                    m.beta_out.copy_(0.02 * torch.randn(m.beta_out.shape, generator=g2))
        qnn.set_quant_state(True, True)
        with torch.no_grad():
            qnn(cali[:8])
        seen, opts, got = [], [], []
        orig_rec, orig_init, orig_gather = BR.LossFunction.record, E.SsqAdam.__init__, BR.K.gather_rows2

        def spy(self, rec, rnd, b):
            r = orig_rec(self, rec, rnd, b)
            seen.append(float(r))
            return r

        def init(self, *a, **k):
            orig_init(self, *a, **k)
            opts.append(self)

        def gather(src0, idx, src1=None, **k):
            got.append(src1 is not None)
            return orig_gather(src0, idx, src1, **k)

        orig_mat = BR.K.A.materialize_rows

        def mat(t):
            if t.data_ptr() in BR.K.A.ROW_VIEWS:
                fallbacks.append(1)
            return orig_mat(t)

        prev = {k: getattr(BR, k) for k in knobs}
        BR.LossFunction.record, E.SsqAdam.__init__, BR.K.gather_rows2 = spy, init, gather
        BR.K.A.materialize_rows = mat
        for k in knobs:
            setattr(BR, k, on and (rows or k != "ROWS_IN_PLACE"))
        try:
            torch.manual_seed(1005)
            Q.block_reconstruction(qnn, block, cali, batch_size=8, iters=12, act_quant=True,
                                   opt_mode="mse", lr=4e-4, p=2.4)
        finally:
            BR.LossFunction.record, E.SsqAdam.__init__, BR.K.gather_rows2 = orig_rec, orig_init, orig_gather
            BR.K.A.materialize_rows = orig_mat
            for k, v in prev.items():
                setattr(BR, k, v)
        out = {"rec": np.array(seen),
               "delta": np.array([float(q.delta) for q in
                                  [block.act_quantizer, block.conv1.act_quantizer,
                                   block.conv2.act_quantizer] if q.delta is not None])}
        for k, o in enumerate(opts):
            for j, p_ in enumerate(o.params):
                out[f"opt{k}_m{j}"] = o.state[p_]["exp_avg"].cpu().numpy()
                out[f"opt{k}_v{j}"] = o.state[p_]["exp_avg_sq"].cpu().numpy()
        runs.append(out)
        pairs.append(sorted(set(got)))
    assert pairs == [[False], [] if rows else [True]], pairs
    assert not fallbacks
    assert runs[0].keys() == runs[1].keys() and len(runs[0]["rec"]) == 12
    for k in runs[0]:
        if k == "rec":
            np.testing.assert_allclose(runs[1][k], runs[0][k], rtol=1e-6, err_msg=k)
        else:
            np.testing.assert_array_equal(runs[1][k], runs[0][k], err_msg=k)


def test_brecq_chunked_loop_bit_identical(Q, golden, det_convs):
    """block_recon.ChunkGraph: after the warm-up, CHUNK_ITERS iterations per graph replay
    (batch draws, schedules and Adam constants staged ahead by one H2D copy, each iteration
    starting with ssq_gather_rows2_staged on its slot) against one iteration per replay:
    AdaRound V / the act delta, Adam's moments, the last loss and the CPU RNG's position
    bit-identical -- BRECQ's per-layer loops (the block's conv1 and the fc, weight phase;
    conv1's act phase), 120 iterations, count-500 boundaries included (the chunk breaks
    before the reported iteration)."""
    import importlib
    BR = importlib.import_module("shiftedscalequantization_amd.quant.block_recon")
    E = importlib.import_module("shiftedscalequantization_amd.quant._engine")
    g = golden("recon_layer_brecq")
    cali = dev(g["cali"])
    runs = []
    for chunk in (1, 25):
        qnn = build_qnn(Q, g)
        layers = [qnn.model[3].conv1, qnn.model[6]]
        opts, orig_init, prev = [], E.SsqAdam.__init__, BR.CHUNK_ITERS

        def init(self, *a, **k):
            orig_init(self, *a, **k)
            opts.append(self)

        E.SsqAdam.__init__, BR.CHUNK_ITERS = init, chunk
        n0 = E.GRAPH_REPLAYS.get("chunk", 0)
        out = {}
        try:
            for k, layer in enumerate(layers):
                torch.manual_seed(1005)
                Q.layer_reconstruction(qnn, layer, cali, batch_size=8, iters=520, weight=0.01,
                                       asym=True, b_range=(20, 2), warmup=0.2, act_quant=False,
                                       opt_mode="mse")
                out[f"w{k}_V"] = layer.weight_quantizer.alpha.detach().cpu().numpy()
            qnn.set_quant_state(True, True)
            with torch.no_grad():
                qnn(cali[:8])
            qnn.disable_network_output_quantization()
            torch.manual_seed(1005)
            Q.layer_reconstruction(qnn, layers[0], cali, batch_size=8, iters=120, act_quant=True,
                                   opt_mode="mse", lr=4e-4, p=2.4)
            out["a_delta"] = np.array([float(layers[0].act_quantizer.delta)])
            out["rng"] = np.array(torch.randint(0, 1 << 30, (4,)).tolist())
            for k, o in enumerate(opts):
                for j, p_ in enumerate(o.params):
                    out[f"opt{k}_m{j}"] = o.state[p_]["exp_avg"].cpu().numpy()
                    out[f"opt{k}_v{j}"] = o.state[p_]["exp_avg_sq"].cpu().numpy()
            out["chunk_replays"] = E.GRAPH_REPLAYS.get("chunk", 0) - n0
        finally:
            E.SsqAdam.__init__, BR.CHUNK_ITERS = orig_init, prev
        runs.append(out)
    assert runs[0]["chunk_replays"] == 0 and runs[1]["chunk_replays"] >= 40, runs[1]["chunk_replays"]
    for k in runs[0]:
        if k != "chunk_replays":
            np.testing.assert_array_equal(runs[1][k], runs[0][k], err_msg=k)


@pytest.mark.parametrize("stage", [False, True])
@pytest.mark.parametrize("affine", [False, True])
def test_brecq_act_chunked_rows_bit_identical(Q, affine, stage, det_convs):
    """BRECQ's act phase on an identity-residual block with the cached rows read in place
    (ROWS_IN_PLACE) and 25 iterations per graph replay: each replayed iteration's first
    launch -- conv1's K13 row-view forward -- copies its ring row into the static words
    (ssq_epilogue_fwd_rows stage_*; no copy launch of its own) and takes its row maps from
    the ring row.  Act deltas, Adam moments and every reported loss bit-identical to one
    iteration per replay; the stage taken by the forward in every chunked iteration (stage) or
    done by a copy launch (the gathering loops' form)."""
    import importlib
    from shiftedscalequantization_amd import nets
    BR = importlib.import_module("shiftedscalequantization_amd.quant.block_recon")
    E = importlib.import_module("shiftedscalequantization_amd.quant._engine")
    A = BR.K.A
    gen = torch.Generator().manual_seed(23)
    cali = torch.randn(32, 3, 12, 12, generator=gen).cuda()
    runs, taken = [], []
    for chunk in (1, 25):
        torch.manual_seed(5)
        net = nn.Sequential(nn.Conv2d(3, 16, 3, padding=1, bias=False), nn.BatchNorm2d(16),
                            nn.ReLU(), nets.BasicBlock(16, 16), nn.AdaptiveAvgPool2d(1),
                            nn.Flatten(), nn.Linear(16, 10)).eval()
        qnn = Q.QuantModel(net, {"n_bits": 2, "channel_wise": True, "scale_method": "max"},
                           {"n_bits": 4, "channel_wise": False, "scale_method": "mse",
                            "leaf_param": True}).cuda().eval()
        qnn.set_first_last_layer_to_8bit()
        block = qnn.model[3]
        if affine:
            g2 = torch.Generator().manual_seed(7)
            for n in ("conv1", "conv2"):
                m = getattr(block, n)
                with torch.no_grad():
                    m.alpha_out.copy_(1 + 0.05 * torch.randn(m.alpha_out.shape, generator=g2))
                    m.beta_out.copy_(0.02 * torch.randn(m.beta_out.shape, generator=g2))
        qnn.set_quant_state(True, True)
        with torch.no_grad():
            qnn(cali[:8])
        seen, opts, took = [], [], [0]
        orig_rec, orig_init, orig_take = BR.LossFunction.record, E.SsqAdam.__init__, A.take_row_stage

        def spy(self, rec, rnd, b, **k):
            r = orig_rec(self, rec, rnd, b, **k)
            seen.append(float(r))
            return r

        def init(self, *a, **k):
            orig_init(self, *a, **k)
            opts.append(self)

        def take():
            st = orig_take()
            took[0] += st is not None
            return st

        prev, prev_st = BR.CHUNK_ITERS, E.BatchFeeder.STAGE_IN_K13
        BR.LossFunction.record, E.SsqAdam.__init__, A.take_row_stage = spy, init, take
        BR.CHUNK_ITERS, E.BatchFeeder.STAGE_IN_K13 = chunk, stage
        n0 = E.GRAPH_REPLAYS.get("chunk", 0)
        try:
            torch.manual_seed(1005)
            Q.block_reconstruction(qnn, block, cali, batch_size=8, iters=120, act_quant=True,
                                   opt_mode="mse", lr=4e-4, p=2.4)
        finally:
            BR.LossFunction.record, E.SsqAdam.__init__, A.take_row_stage = orig_rec, orig_init, orig_take
            BR.CHUNK_ITERS, E.BatchFeeder.STAGE_IN_K13 = prev, prev_st
        out = {"rec": np.array(seen),
               "delta": np.array([float(q.delta) for q in
                                  [block.act_quantizer, block.conv1.act_quantizer,
                                   block.conv2.act_quantizer] if q.delta is not None])}
        for k, o in enumerate(opts):
            for j, p_ in enumerate(o.params):
                out[f"opt{k}_m{j}"] = o.state[p_]["exp_avg"].cpu().numpy()
                out[f"opt{k}_v{j}"] = o.state[p_]["exp_avg_sq"].cpu().numpy()
        runs.append(out)
        taken.append((took[0], E.GRAPH_REPLAYS.get("chunk", 0) - n0))
    # chunk 25: the stage is taken once per captured iteration (the graph holds 25) and the
    # loop replays the chunk graph at least 4 times (120 iterations after a 4-iteration warm-up)
    assert taken[0] == (0, 0) and taken[1][0] == (25 if stage else 0) and taken[1][1] >= 4, taken
    assert runs[0].keys() == runs[1].keys()
    bad = np.nonzero(runs[1]["rec"] != runs[0]["rec"])[0]
    assert bad.size == 0, ("iterations whose loss differs", bad.tolist())
    for k in runs[0]:
        np.testing.assert_array_equal(runs[1][k], runs[0][k], err_msg=k)


@pytest.mark.parametrize("bits", [4, 8])
def test_fc_fused_iteration_matches_unfused(Q, det_convs, bits):
    """K19 (kernels.fc_recon_iter, block_recon.FUSE_FC): BRECQ's layer loop on a Linear
    layer at ResNet-18's fc shape (512 -> 1000, 8-bit AdaRound, batch 32), the iteration as
    two launches (AdaRound forward on the fly + GEMM + bias + p = 2 loss and gradient; dW +
    AdaRound backward with the rounding regulariser + Adam) against the unfused launches:
    every iteration's loss to 1e-5, V walk-bounded (the GEMMs' fp32 summation order is not
    hipBLASLt's: entries whose gradient is at that order's noise floor take Adam's +-lr steps
    either way), hard-rounding decisions flipped only inside the walk budget.  At 8 bits the
    loss is a sum of squares of y - t ~ 1e-3 |y| (observed r5: loss ~1e-5): a 1e-7 relative
    difference of y between the two GEMM orders is ~1e-4 of the loss (observed max 4.7e-5),
    so the 8-bit case is held at 1e-4.  For the same reason most 8-bit V gradients sit at the
    GEMM-order noise floor, where Adam's normalised step is +-lr whichever sign the noise
    takes: r5 saw 4.3 % of V entries walk (max 0.022, inside the 0.6 walk budget), so at 8 bits
    the walk is held to its budget and the per-step agreement is pinned where it is
    deterministic -- test_fc_recon_iter_vs_reference (one iteration at this shape against
    float64 dW / y, Adam bit-identical); 4 bits keeps the 1 % walker bound."""
    import copy
    import importlib
    from conftest import assert_hard_flips_bounded as ahf
    BR = importlib.import_module("shiftedscalequantization_amd.quant.block_recon")
    torch.manual_seed(11)
    lin = nn.Linear(512, 1000)
    cali = torch.relu(torch.randn(256, 512)).cuda()
    iters = 300
    runs, orig_rec, orig_init, orig_fc = [], BR.LossFunction.record, BR.LossFunction.__init__, BR.K.fc_recon_iter
    for fuse in (False, True):
        qnn = Q.QuantModel(nn.Sequential(copy.deepcopy(lin)), {"n_bits": bits, "channel_wise": True, "scale_method": "max"},
                           {"n_bits": 8, "channel_wise": False, "scale_method": "max"}).cuda().eval()
        qnn.set_quant_state(True, False)
        with torch.no_grad():
            qnn(cali[:64])
        fc = [m for m in qnn.modules() if isinstance(m, Q.QuantModule)][-1]
        seen, calls = [], []

        def spy(self, rec, rnd, b, **k):
            r = orig_rec(self, rec, rnd, b, **k)
            seen.append(float(r))
            return r

        def init(self, *a, **k):
            orig_init(self, *a, **k)
            self.track_values = True

        def fcs(*a, **k):
            calls.append(1)
            return orig_fc(*a, **k)

        prev = BR.FUSE_FC
        BR.LossFunction.record, BR.LossFunction.__init__, BR.K.fc_recon_iter, BR.FUSE_FC = spy, init, fcs, fuse
        try:
            torch.manual_seed(1005)
            Q.layer_reconstruction(qnn, fc, cali, batch_size=32, iters=iters, weight=0.01, asym=True,
                                   b_range=(20, 2), warmup=0.2, act_quant=False, opt_mode="mse")
        finally:
            BR.LossFunction.record, BR.LossFunction.__init__, BR.K.fc_recon_iter, BR.FUSE_FC = \
                orig_rec, orig_init, orig_fc, prev
        q = fc.weight_quantizer
        v = q.alpha.detach().cpu().numpy()
        q.soft_targets = False
        with torch.no_grad():
            what = q(fc.weight).cpu().numpy()
        runs.append((np.array(seen), v, what, len(calls)))
    (l0, v0, w0, c0), (l1, v1, w1, c1) = runs
    assert c0 == 0 and c1 >= 1, (c0, c1)        # host calls: the eager warm-up + one capture
    stats = {"loss_rel_err": np.max(np.abs(l1 - l0) / np.abs(l0)), "loss_min": float(l0.min())}
    np.testing.assert_allclose(l1, l0, rtol=1e-5 if bits == 4 else 1e-4)
    dv = np.abs(v1 - v0)
    stats["V_dev"] = dv.max()
    if bits == 4:
        stats["V_walkers"] = assert_walk_bounded(dv, 1e-5, iters * 2e-3, frac=0.01, what="fc V")
    else:
        stats["V_walkers"] = int((dv > 1e-5).sum())
        assert dv.max() <= iters * 2e-3, dv.max()
    stats["hard_flips"] = ahf(w1, w0, v1, v0, iters * 2e-3, "fc")
    parity_report(f"k19_fc_fused_vs_unfused[w{bits}]", **stats)


def fc_mlp():
    """make_golden.gen_recon_layer_brecq_fc's network (weights from the fixture)."""
    return nn.Sequential(nn.Linear(64, 512), nn.ReLU(), nn.Linear(512, 40)).eval()


def fc_slot(bs, perm, lam, b, step):
    """The device words of BRECQ iteration `step` (0-based) as BatchFeeder stages them: the
    batch indices, (lambda, b), Adam's (-lr/bc1, sqrt(bc2)) at lr 1e-3, betas (0.9, 0.999)."""
    slot = torch.zeros(bs + 2, dtype=torch.int64)
    slot[:bs] = torch.as_tensor(perm.astype(np.int64))
    t = step + 1
    words = np.array([lam, b, -1e-3 / (1 - 0.9 ** t), (1 - 0.999 ** t) ** 0.5], np.float32)
    slot[bs:] = torch.from_numpy(words.view(np.int64))
    return slot.cuda()


def test_fc_loop_matches_reference(Q, golden):
    """K19, the fc loop as production runs it (FUSE_FC, CHUNK_ITERS iterations per graph
    replay, no per-iteration value tracking), against the reference's own trajectory
    (recon_layer_brecq_fc.npz: layer_reconstruction, quant/layer_recon.py:10-104, on an
    8-bit Linear(512, 40) -- C_in % 64 == 0, so K19 is taken; 40 outputs leave a partial
    16-row tile as ResNet-18's 1000 do -- 200 iterations over the b schedule's warm-up,
    decay and end).  The captured input / target are the reference's (teacher-forced: the
    first layer's GEMM order is not the loop under test; ours is checked against them too).
      * every batch draw identical;
      * every iteration's rec loss within max(1e-5, 2x the reference's own largest
        distance from float64) of the reference's, and as close to the float64 loss as the
        reference is (2x) -- at 8 bits the loss is a sum of squares of y - t ~ 4e-3 |y|,
        so a GEMM's fp32 summation order moves it by ~1e-5 (the reference's own distance
        from float64: max 9.5e-6, median 2.2e-6);
      * V walk-bounded, hard rounding flipped only inside the walk budget;
      * teacher-forced V gradients at steps 0 / 45 / 199 (K19's gv_out at the reference's V
        and batch) within 2x the reference's own distance from the float64 gradient."""
    import importlib
    from conftest import assert_hard_flips_bounded as ahf
    BR = importlib.import_module("shiftedscalequantization_amd.quant.block_recon")
    E = importlib.import_module("shiftedscalequantization_amd.quant._engine")
    g = golden("recon_layer_brecq_fc")
    iters, bs = int(g["iters"][0]), int(g["bs"][0])
    qnn = build_qnn(Q, g, net=fc_mlp())
    fc = [m for m in qnn.modules() if isinstance(m, Q.QuantModule)][-1]
    assert fc.weight_quantizer.n_bits == 8 and tuple(fc.weight.shape) == (40, 512)
    cali = dev(g["cali"])
    seen, draws, calls, cap = [], [], [], {}
    orig = (BR.LossFunction.record, BR.K.fc_recon_iter, BR.save_inp_oup_data, E.BatchFeeder.draw)

    def spy(self, rec, rnd, b, count=None):
        seen.append((self.count if count is None else count, float(rec)))
        return orig[0](self, rec, rnd, b, count=count)

    def fcs(*a, **k):
        calls.append(1)
        return orig[1](*a, **k)

    def save_io(*a, **k):
        inp, out = orig[2](*a, **k)
        cap["inp_rel"] = (inp.cpu().numpy() - g["cached_inp"]).__abs__().max() / np.abs(g["cached_inp"]).max()
        cap["out_rel"] = (out.cpu().numpy() - g["cached_out"]).__abs__().max() / np.abs(g["cached_out"]).max()
        return dev(g["cached_inp"]), dev(g["cached_out"])

    def draw(self):
        p = orig[3](self)
        draws.append(p.numpy().copy())
        return p

    BR.LossFunction.record, BR.K.fc_recon_iter, BR.save_inp_oup_data, E.BatchFeeder.draw = \
        spy, fcs, save_io, draw
    n0 = E.GRAPH_REPLAYS.get("chunk", 0)
    try:
        assert BR.FUSE_FC and BR.CHUNK_ITERS > 1, "production knobs"
        torch.manual_seed(1005)
        Q.layer_reconstruction(qnn, fc, cali, batch_size=bs, iters=iters, weight=0.01, asym=True,
                               b_range=(20, 2), warmup=0.2, act_quant=False, opt_mode="mse")
    finally:
        BR.LossFunction.record, BR.K.fc_recon_iter, BR.save_inp_oup_data, E.BatchFeeder.draw = orig
    chunks = E.GRAPH_REPLAYS.get("chunk", 0) - n0
    # K19 engaged (the eager warm-up calls, one single-iteration capture, one chunk capture)
    # and the loop ran on chunk replays
    assert len(calls) >= 2 and chunks >= 5, (len(calls), chunks)
    # our capture of the same input / target: the first layer's GEMM order only
    assert cap["inp_rel"] <= 1e-6 and cap["out_rel"] <= 1e-6, cap
    np.testing.assert_array_equal(np.stack(draws), g["perms"].astype(np.int64))
    assert [c for c, _ in seen] == list(range(1, iters + 1))
    rec = np.array([v for _, v in seen])
    ref, ref64 = g["rec_loss"], g["rec_loss64"]
    rel = np.abs(rec - ref) / np.abs(ref)
    ref_self = np.abs(ref - ref64) / np.abs(ref64)
    our_self = np.abs(rec - ref64) / np.abs(ref64)
    stats = {"loss_rel_err": rel.max(), "loss_rel_median": np.median(rel),
             "ref_vs_f64_max": ref_self.max(), "ours_vs_f64_max": our_self.max(),
             "ours_vs_f64_median": np.median(our_self), "ref_vs_f64_median": np.median(ref_self),
             "chunk_replays": chunks, "capture_inp_rel": cap["inp_rel"]}
    q = fc.weight_quantizer
    v = q.alpha.detach().cpu().numpy()
    dv = np.abs(v - g["V"])
    stats["V_dev"] = dv.max()
    stats["V_walkers"] = int((dv > 1e-5).sum())
    q.soft_targets = False
    with torch.no_grad():
        what = q(fc.weight).cpu().numpy()
    d, z = g["qm1_delta"][:, None], g["qm1_zp"][:, None]
    what_ref = (g["what_hard_codes"].astype(np.float32) - z) * d
    stats["hard_flips"] = ahf(what, what_ref, v, g["V"], iters * 2e-3, "fc")
    # teacher-forced V gradients
    w = fc.weight.detach().contiguous()
    dq, zq = q.delta.detach(), q.zero_point.detach()
    decay = BR.LinearTempDecay(iters, rel_start_decay=0.2, start_b=20, end_b=2)
    for s in g["grad_steps"]:
        s = int(s)
        V = dev(g[f"gs{s}_V"]).contiguous()
        lam = 0.01 if (s + 1) >= 0.2 * iters else 0.0
        slot = fc_slot(bs, g["perms"][s], lam, float(decay(s + 1)) if lam else 0.0, s)
        what_s = K_adaround(Q, V, w, dq, zq)
        gv = torch.empty_like(V)
        m_, v_ = torch.zeros_like(V), torch.zeros_like(V)
        BR.K.fc_recon_iter(dev(g["cached_inp"]), dev(g["cached_out"]), slot, bs, w, V.clone(),
                           what_s, dq, zq, 8, fc.bias.detach(), m_, v_, 0.9, 0.999, 1e-8, gv_out=gv)
        gr = g[f"gs{s}_g"].astype(np.float64)
        truth = gr + g[f"gs{s}_t_minus_g"].astype(np.float64)
        ours = np.abs(gv.cpu().numpy().astype(np.float64) - truth).max()
        theirs = np.abs(gr - truth).max()
        stats[f"gs{s}_ours_vs_f64"], stats[f"gs{s}_ref_vs_f64"] = ours, theirs
        stats[f"gs{s}_maxabs"] = np.abs(truth).max()
    parity_report("k19_fc_loop_vs_reference", **stats)
    tol = max(1e-5, 2 * ref_self.max())
    assert rel.max() <= tol, (rel.max(), tol, int(rel.argmax()))
    assert our_self.max() <= 2 * ref_self.max(), (our_self.max(), ref_self.max())
    assert_walk_bounded(dv, 1e-5, iters * 2e-3, frac=0.05, what="fc V")
    for s in g["grad_steps"]:
        assert stats[f"gs{s}_ours_vs_f64"] <= 2 * stats[f"gs{s}_ref_vs_f64"], \
            (int(s), stats[f"gs{s}_ours_vs_f64"], stats[f"gs{s}_ref_vs_f64"])


def K_adaround(Q, V, w, d, z):
    """W^ = AdaRound's soft forward (ssq_adaround_fwd), the first K19 call's input."""
    from shiftedscalequantization_amd import kernels as K
    return K.adaround(V, w, d, z, 8, False, False).detach().clone()


@pytest.mark.parametrize("shape", [(512, 1000), (512, 40)])
def test_fc_chunked_loop_bit_identical(Q, det_convs, shape):
    """The production fc loop -- K19 inside ChunkGraph replays, track_values off, so the
    iteration reads its words straight from the chunk ring row (feeder.chunk_dev[slot]) --
    against one iteration per replay (CHUNK_ITERS = 1): V, Adam's moments, every recorded
    rec loss and the CPU RNG's position bit-identical, at ResNet-18's fc shape (512 -> 1000)
    and the fixture's (512 -> 40)."""
    import copy
    import importlib
    BR = importlib.import_module("shiftedscalequantization_amd.quant.block_recon")
    E = importlib.import_module("shiftedscalequantization_amd.quant._engine")
    ci, co = shape
    torch.manual_seed(11)
    lin = nn.Linear(ci, co)
    cali = torch.relu(torch.randn(256, ci)).cuda()
    runs = []
    for chunk in (1, 25):
        qnn = Q.QuantModel(nn.Sequential(copy.deepcopy(lin)),
                           {"n_bits": 8, "channel_wise": True, "scale_method": "max"},
                           {"n_bits": 8, "channel_wise": False, "scale_method": "max"}).cuda().eval()
        qnn.set_quant_state(True, False)
        with torch.no_grad():
            qnn(cali[:64])
        fc = [m for m in qnn.modules() if isinstance(m, Q.QuantModule)][-1]
        seen, opts, calls = [], [], []
        orig_rec, orig_init, orig_fc, prev = (BR.LossFunction.record, E.SsqAdam.__init__,
                                              BR.K.fc_recon_iter, BR.CHUNK_ITERS)

        def spy(self, rec, rnd, b, count=None):
            seen.append(float(rec))
            return orig_rec(self, rec, rnd, b, count=count)

        def init(self, *a, **k):
            orig_init(self, *a, **k)
            opts.append(self)

        def fcs(*a, **k):
            calls.append(1)
            return orig_fc(*a, **k)

        BR.LossFunction.record, E.SsqAdam.__init__, BR.K.fc_recon_iter, BR.CHUNK_ITERS = \
            spy, init, fcs, chunk
        n0 = E.GRAPH_REPLAYS.get("chunk", 0)
        try:
            torch.manual_seed(1005)
            Q.layer_reconstruction(qnn, fc, cali, batch_size=32, iters=160, weight=0.01,
                                   asym=True, b_range=(20, 2), warmup=0.2, act_quant=False,
                                   opt_mode="mse")
        finally:
            BR.LossFunction.record, E.SsqAdam.__init__, BR.K.fc_recon_iter, BR.CHUNK_ITERS = \
                orig_rec, orig_init, orig_fc, prev
        out = {"rec": np.array(seen), "V": fc.weight_quantizer.alpha.detach().cpu().numpy(),
               "rng": np.array(torch.randint(0, 1 << 30, (4,)).tolist()),
               "replays": E.GRAPH_REPLAYS.get("chunk", 0) - n0, "fused": len(calls)}
        for j, p_ in enumerate(opts[0].params):
            out[f"m{j}"] = opts[0].state[p_]["exp_avg"].cpu().numpy()
            out[f"v{j}"] = opts[0].state[p_]["exp_avg_sq"].cpu().numpy()
        runs.append(out)
    assert runs[0]["replays"] == 0 and runs[1]["replays"] >= 5, runs[1]["replays"]
    assert runs[0]["fused"] >= 2 and runs[1]["fused"] >= 2
    assert len(runs[0]["rec"]) == len(runs[1]["rec"]) == 160
    for k in runs[0]:
        if k not in ("replays", "fused"):
            np.testing.assert_array_equal(runs[1][k], runs[0][k], err_msg=k)


def test_brecq_frozen_loop_skips_unreported_iterations(Q, golden):
    """A loop in which nothing learns (the fc's act phase: its act quantizer is the disabled
    network output) runs only its reported iterations (SKIP_FROZEN): the same printed
    losses (every 500th count, and the last), the same final state, and the CPU RNG left
    where the full loop leaves it (the reference draws a randperm every iteration)."""
    import importlib
    BR = importlib.import_module("shiftedscalequantization_amd.quant.block_recon")
    g = golden("recon_layer_brecq")
    cali = dev(g["cali"])
    runs = []
    for skip in (False, True):
        qnn = build_qnn(Q, g)
        fc = qnn.model[6]
        qnn.set_quant_state(True, True)
        with torch.no_grad():
            qnn(cali[:8])
        qnn.disable_network_output_quantization()
        reported, orig_rec, prev = [], BR.LossFunction.record, BR.SKIP_FROZEN

        def spy(self, rec, rnd, b):
            r = orig_rec(self, rec, rnd, b)
            if self.count % 500 == 0 or self.count == 1001:
                reported.append((self.count, float(r)))
            return r

        BR.LossFunction.record, BR.SKIP_FROZEN = spy, skip
        try:
            torch.manual_seed(1005)
            Q.layer_reconstruction(qnn, fc, cali, batch_size=8, iters=1001, act_quant=True,
                                   opt_mode="mse", lr=4e-4, p=2.4)
            nxt = torch.randint(0, 1 << 30, (4,)).tolist()
        finally:
            BR.LossFunction.record, BR.SKIP_FROZEN = orig_rec, prev
        runs.append((reported, nxt, float(fc.act_quantizer.delta)))
    assert [c for c, _ in runs[0][0]] == [500, 1000, 1001]
    assert runs[0] == runs[1]


# ------------------------------------------------------------------ other block types
def block_net(kind):
    from shiftedscalequantization_amd import nets
    if kind == "bottleneck":
        ds = nn.Sequential(nn.Conv2d(16, 32, 1, stride=2, bias=False), nn.BatchNorm2d(32))
        blk, cout = nets.Bottleneck(16, 8, stride=2, downsample=ds), 32
    elif kind == "inverted":
        blk, cout = nets.InvertedResidual(16, 16, 1, 2), 16
    else:
        blk, cout = nets.ResBottleneckBlock(16, 32, 2, 8), 32
    return nn.Sequential(nn.Conv2d(3, 16, 3, padding=1, bias=False), nn.BatchNorm2d(16), nn.ReLU(),
                         blk, nn.AdaptiveAvgPool2d(1), nn.Flatten(), nn.Linear(cout, 10)).eval()


def block_qnn(Q, kind):
    wq = {"n_bits": 2, "channel_wise": True, "scale_method": "max"}
    aq = {"n_bits": 4, "channel_wise": False, "scale_method": "mse", "leaf_param": True}
    qnn = Q.QuantModel(block_net(kind), wq, aq).cuda().eval()
    qnn.set_first_last_layer_to_8bit()
    return qnn


def named_qms(block, Q):
    return [(n, m) for n, m in block.named_modules() if isinstance(m, Q.QuantModule)]


def set_module(Q, m, w, b, d, z, bits=2):
    w, b = dev(w), dev(b)
    m.org_weight, m.org_bias = w.clone(), b.clone()
    m.weight.data = w.clone()
    m.bias = nn.Parameter(b.clone())
    uaq = Q.UniformAffineQuantizer(n_bits=bits, channel_wise=True, ch=w.shape).cuda()
    shape = (-1,) + (1,) * (w.dim() - 1)
    uaq.delta = nn.Parameter(dev(d).view(shape))
    uaq.zero_point = nn.Parameter(dev(z).view(shape))
    uaq.inited = True
    return uaq


@pytest.mark.parametrize("kind", ["bottleneck", "inverted", "resbottleneck"])
def test_fused_recon_other_blocks_match_reference(Q, golden, kind):
    """block_recon_fused_shiftedScale on a ResNet-50 Bottleneck, a MobileNetV2
    InvertedResidual (depthwise conv: alpha (1, S)) and a RegNetX ResBottleneck (grouped
    conv) against the reference's own trajectory (tests/golden/recon_block_<kind>.npz)."""
    g = golden(f"recon_block_{kind}")
    qnn = block_qnn(Q, kind)
    block = qnn.model[3]
    for n, m in named_qms(block, Q):
        uaq = set_module(Q, m, g[f"f_{n}_w"], g[f"f_{n}_b"], g[f"f_{n}_delta"], g[f"f_{n}_zp"])
        m.weight_quantizer = Q.ChannelQuant(1.0, uaq=uaq, weight_tensor=m.org_weight, shiftTarget=SHIFTS,
                                            name="." + n)
        m.use_weight_quant = True
    block.cached_inp_features = [dev(g["f_cached_inp"])]
    block.cached_out_features = [dev(g["f_cached_out"])]
    iters = int(g["iters"][0])
    import importlib
    LRF = importlib.import_module("shiftedscalequantization_amd.quant.layer_recon_fused_shiftedScale")
    seen_perms, seen_rec = [], []
    orig_draw, orig_keep = LRF.BatchFeeder.draw, LRF.FusedScaleLossFunction.bookkeep

    def draw(self):
        p = orig_draw(self)
        seen_perms.append(p.clone())
        return p

    def bookkeep(self, rec):
        seen_rec.append(float(rec.item()))
        return orig_keep(self, rec)

    LRF.BatchFeeder.draw, LRF.FusedScaleLossFunction.bookkeep = draw, bookkeep
    try:
        torch.manual_seed(1005)
        res = LRF.block_recon_fused_shiftedScale(block, iters, (0.01, 0.1), qnn, None, verbose=False)
    finally:
        LRF.BatchFeeder.draw, LRF.FusedScaleLossFunction.bookkeep = orig_draw, orig_keep
    np.testing.assert_array_equal(np.stack([p.numpy() for p in seen_perms]), g["f_perms"])
    stats = {"rec_rel_err": np.max(np.abs(np.array(seen_rec) - g["f_rec_loss"][:iters]) /
                                   np.abs(g["f_rec_loss"][:iters])),
             "final_rel_err": np.max(np.abs(np.array(res) - g["f_final_losses"]) / np.abs(g["f_final_losses"]))}
    # observed (r2): rel errs <= 6.4e-7, non-walking alpha rows <= 7.3e-6, 0 hard flips
    np.testing.assert_allclose(seen_rec, g["f_rec_loss"][:iters], rtol=1e-5)
    np.testing.assert_allclose(res, g["f_final_losses"], rtol=1e-5)
    from oracle import ssq_ref as R
    for n, m in named_qms(block, Q):
        q = m.weight_quantizer
        w = g[f"f_{n}_w"]
        fl = np.stack(R.shift_floors(w, g[f"f_{n}_delta"].reshape(-1, 1, 1, 1), SHIFTS))
        degenerate = np.all(fl == fl[:1], axis=(0, 1, 3, 4))
        da = np.abs(q.alpha.detach().cpu().numpy() - g[f"f_{n}_alpha"])
        # Besides exactly degenerate rows (zero analytic gradient), a row whose gradient is
        # a near-total cancellation is noise-dominated: Adam turns the sign of the residue
        # into +-lr steps, in the reference as here.  At most ~10 % of a layer's rows (at
        # least one) may take such a walk, bounded by iters * 2 * lr; every other row
        # follows the reference trajectory to 2e-4.
        off = ~degenerate & (da.max(axis=-1) > 2e-4)
        stats[n + "_walking_rows"] = off.sum()
        stats[n + "_rows"] = off.size
        stats[n + "_alpha_dev_other"] = da[~degenerate & ~off].max(initial=0.0)
        assert off.sum() <= max(1, round(0.1 * off.size)), (n, np.nonzero(off)[0], da.max())
        assert da.max(initial=0.0) <= iters * 1e-3 * 2, n
        with torch.no_grad():
            what = q(m.weight).cpu().numpy()
        stats[n + "_hard_flips"] = assert_shift_flips_bounded(
            what, g[f"f_{n}_what_hard"], q.alpha.detach().cpu().numpy(), g[f"f_{n}_alpha"],
            iters * 2e-3, n)
        stats[n + "_n"] = what.size
        assert stats[n + "_alpha_dev_other"] <= 5e-5, n
    parity_report(f"a18_fused_{kind}", **stats)


@pytest.mark.parametrize("kind", ["bottleneck", "inverted", "resbottleneck"])
def test_brecq_other_blocks_match_reference(Q, golden, kind):
    """BRECQ AdaRound block reconstruction on the same three block types against the
    reference's per-iteration total losses and final AdaRound alphas."""
    g = golden(f"recon_block_{kind}")
    qnn = block_qnn(Q, kind)
    qms = [m for m in qnn.modules() if isinstance(m, Q.QuantModule)]
    for k, m in enumerate(qms):
        bits = 8 if k in (0, len(qms) - 1) else 2
        m.weight_quantizer = set_module(Q, m, g[f"b_qm{k}_w"], g[f"b_qm{k}_b"], g[f"b_qm{k}_delta"],
                                        g[f"b_qm{k}_zp"], bits)
    block = qnn.model[3]
    cali = dev(g["b_cali"])
    import importlib
    BR = importlib.import_module("shiftedscalequantization_amd.quant.block_recon")
    seen = []
    orig_rec, orig_init = BR.LossFunction.record, BR.LossFunction.__init__

    def spy(self, rec, rnd, b):
        r = orig_rec(self, rec, rnd, b)
        seen.append(float(r))
        return r

    def init(self, *a, **k):
        orig_init(self, *a, **k)
        self.track_values = True

    BR.LossFunction.record, BR.LossFunction.__init__ = spy, init
    try:
        torch.manual_seed(1005)
        Q.block_reconstruction(qnn, block, cali, batch_size=8, iters=int(g["iters"][1]), weight=0.01,
                               asym=True, b_range=(20, 2), warmup=0.2, act_quant=False, opt_mode="mse")
    finally:
        BR.LossFunction.record, BR.LossFunction.__init__ = orig_rec, orig_init
    stats = {"total_rel_err": np.max(np.abs(np.array(seen) - g["b_total_loss"]) / np.abs(g["b_total_loss"]))}
    np.testing.assert_allclose(seen, g["b_total_loss"], rtol=1e-5)      # observed <= 1.6e-7
    iters = int(g["iters"][1])
    for n, m in named_qms(block, Q):
        q = m.weight_quantizer
        dv = np.abs(q.alpha.detach().cpu().numpy() - g[f"b_{n}_alpha"])
        stats[n + "_V_dev"] = dv.max()
        stats[n + "_V_walkers"] = int((dv > 1e-5).sum())
        # observed <= 2.4e-6 on most boxes; an entry whose gradient nearly cancels can be
        # walked by Adam (lr 1e-3) in the fp32 summation order of the box's conv solvers
        # (one of 512 by 1.5e-5 on one box): a handful of entries, within Adam's budget
        assert_walk_bounded(dv, 1e-5, iters * 2e-3, what=n)
        with torch.no_grad():
            what = q(m.weight).cpu().numpy()
        stats[n + "_hard_flips"] = assert_hard_flips_bounded(
            what, g[f"b_{n}_what_hard"], q.alpha.detach().cpu().numpy(), g[f"b_{n}_alpha"],
            iters * 2e-3, n)
    parity_report(f"a22_brecq_{kind}", **stats)


@pytest.mark.parametrize("graph", [False, True])
def test_deferred_finalize_bit_identical(Q, golden, graph, det_convs):
    """The fused loop with bias_cal queues its loss and gamma^z/phi^z finalizes onto the next
    backward launch (csrc/fin_tasks.h): alpha, gamma^z, phi^z and every iteration's loss
    are bit-identical to the loop that launches each finalize on its own."""
    import importlib
    LRF = importlib.import_module("shiftedscalequantization_amd.quant.layer_recon_fused_shiftedScale")
    g = golden("recon_fused")
    runs = []
    for defer in (False, True):
        qnn = build_qnn(Q, {})
        block = qnn.model[3]
        load_block(Q, g, block)
        block.cached_inp_features = [dev(g["cached_inp"])]
        block.cached_out_features = [dev(g["cached_out"])]
        seen = []
        orig_keep = LRF.FusedScaleLossFunction.bookkeep

        def bookkeep(self, rec):
            seen.append(float(rec.item()))
            return orig_keep(self, rec)

        LRF.FusedScaleLossFunction.bookkeep, prev = bookkeep, LRF.DEFER_FINALIZE
        LRF.DEFER_FINALIZE = defer
        try:
            torch.manual_seed(1005)
            res = LRF.block_recon_fused_shiftedScale(block, 12, (0.01, 0.1), qnn, None, verbose=False,
                                                     graph=graph, bias_cal=True)
        finally:
            LRF.FusedScaleLossFunction.bookkeep, LRF.DEFER_FINALIZE = orig_keep, prev
        out = {"rec": np.array(seen), "final": np.array(res)}
        for n in ("conv1", "conv2", "downsample"):
            m = getattr(block, n)
            out[n + "_alpha"] = m.weight_quantizer.alpha.detach().cpu().numpy()
            out[n + "_gamma"] = m.alpha_out.detach().cpu().numpy()
            out[n + "_phi"] = m.beta_out.detach().cpu().numpy()
        runs.append(out)
    for k in runs[0]:
        np.testing.assert_array_equal(runs[1][k], runs[0][k], err_msg=k)
    # gamma^z / phi^z really were learned (their finalizes ran)
    assert any(np.any(runs[1][n + "_gamma"] != 1.0) for n in ("conv1", "conv2", "downsample"))


@pytest.mark.parametrize("graph", [False, True])
def test_fused_start_bit_identical(Q, golden, graph, det_convs):
    """The iteration start as one launch (every conv's prepared What riding on the batch
    gather, K.deferred_prep_fwd / csrc/prep_ride.h) against the two launches: every
    iteration's loss and the learned alpha, gamma^z, phi^z bit-identical."""
    import importlib
    LRF = importlib.import_module("shiftedscalequantization_amd.quant.layer_recon_fused_shiftedScale")
    g = golden("recon_fused")
    runs = []
    for fuse in (False, True):
        qnn = build_qnn(Q, {})
        block = qnn.model[3]
        load_block(Q, g, block)
        block.cached_inp_features = [dev(g["cached_inp"])]
        block.cached_out_features = [dev(g["cached_out"])]
        seen = []
        orig_keep = LRF.FusedScaleLossFunction.bookkeep

        def bookkeep(self, rec):
            seen.append(float(rec.item()))
            return orig_keep(self, rec)

        LRF.FusedScaleLossFunction.bookkeep, prev = bookkeep, LRF.FUSE_START
        LRF.FUSE_START = fuse
        try:
            torch.manual_seed(1005)
            LRF.block_recon_fused_shiftedScale(block, 12, (0.01, 0.1), qnn, None, verbose=False,
                                               graph=graph, bias_cal=True)
        finally:
            LRF.FusedScaleLossFunction.bookkeep, LRF.FUSE_START = orig_keep, prev
        out = {"rec": np.array(seen)}
        for n in ("conv1", "conv2", "downsample"):
            m = getattr(block, n)
            out[n + "_alpha"] = m.weight_quantizer.alpha.detach().cpu().numpy()
            out[n + "_gamma"] = m.alpha_out.detach().cpu().numpy()
        runs.append(out)
    for k in runs[0]:
        np.testing.assert_array_equal(runs[1][k], runs[0][k], err_msg=k)


@pytest.mark.parametrize("graph", [False, True])
@pytest.mark.parametrize("bias_cal", [False, True])
def test_fused_adam_bit_identical(Q, golden, graph, bias_cal, det_convs):
    """The optimizer step armed into the alpha backward's launch (SsqAdam.arm: alpha updated
    in its finaliser, gamma^z / phi^z in their finalize tasks or extra workgroups) against
    the separate ssq_adam launch: every iteration's loss, the learned parameters and Adam's
    moments bit-identical; the armed step really ran inside the launch."""
    import importlib
    from shiftedscalequantization_amd.quant import _engine as E
    LRF = importlib.import_module("shiftedscalequantization_amd.quant.layer_recon_fused_shiftedScale")
    g = golden("recon_fused")
    runs, taken, took = [], [], []
    orig_step = E.SsqAdam.step
    orig_take = E.K.adam_take

    def step(self, hyper=None):
        taken.append(bool(getattr(self, "_armed", False)))
        return orig_step(self, hyper)

    def take(device=None):
        r = orig_take(device)
        took.append(bool(r))     # True: the armed step really ran inside the alpha launch
        return r

    for fuse in (False, True):
        qnn = build_qnn(Q, {})
        block = qnn.model[3]
        load_block(Q, g, block)
        block.cached_inp_features = [dev(g["cached_inp"])]
        block.cached_out_features = [dev(g["cached_out"])]
        seen, opts = [], []
        orig_keep = LRF.FusedScaleLossFunction.bookkeep
        orig_init = E.SsqAdam.__init__

        def bookkeep(self, rec):
            seen.append(float(rec.item()))
            return orig_keep(self, rec)

        def init(self, *a, **k):
            orig_init(self, *a, **k)
            opts.append(self)

        LRF.FusedScaleLossFunction.bookkeep, prev = bookkeep, LRF.FUSE_ADAM
        E.SsqAdam.__init__, E.SsqAdam.step = init, step
        E.K.adam_take = take
        LRF.FUSE_ADAM = fuse
        taken.clear()
        took.clear()
        try:
            torch.manual_seed(1005)
            LRF.block_recon_fused_shiftedScale(block, 12, (0.01, 0.1), qnn, None, verbose=False,
                                               graph=graph, bias_cal=bias_cal)
        finally:
            LRF.FusedScaleLossFunction.bookkeep, LRF.FUSE_ADAM = orig_keep, prev
            E.SsqAdam.__init__, E.SsqAdam.step = orig_init, orig_step
            E.K.adam_take = orig_take
        assert any(taken) == fuse
        # every step() that ran on the host (eager iterations and the graph capture) found
        # its armed update already applied by the alpha backward's launch
        assert len(took) == sum(taken)
        if fuse:
            assert took and all(took), took
        out = {"rec": np.array(seen)}
        for n in ("conv1", "conv2", "downsample"):
            m = getattr(block, n)
            out[n + "_alpha"] = m.weight_quantizer.alpha.detach().cpu().numpy()
            out[n + "_gamma"] = m.alpha_out.detach().cpu().numpy()
            out[n + "_phi"] = m.beta_out.detach().cpu().numpy()
        for k, p_ in enumerate(opts[0].params):
            out[f"m{k}"] = opts[0].state[p_]["exp_avg"].cpu().numpy()
            out[f"v{k}"] = opts[0].state[p_]["exp_avg_sq"].cpu().numpy()
        runs.append(out)
    assert runs[0].keys() == runs[1].keys()
    for k in runs[0]:
        np.testing.assert_array_equal(runs[1][k], runs[0][k], err_msg=k)
    if bias_cal:
        assert any(np.any(runs[1][n + "_gamma"] != 1.0) for n in ("conv1", "conv2", "downsample"))


@pytest.mark.parametrize("graph", [False, True])
def test_fused_tail_matches_unfused(Q, golden, graph, det_convs):
    """The block's final epilogue + the p = 2 loss + the epilogue backward as one pass
    (K.epilogue_loss_bwd, the loop's FUSE_TAIL) against the three separate launches: every
    learned parameter (alpha, gamma^z, phi^z) bit-identical after the loop, per-iteration
    losses equal to the last float ulps (row-wise vs block-wise loss partials)."""
    import importlib
    LRF = importlib.import_module("shiftedscalequantization_amd.quant.layer_recon_fused_shiftedScale")
    g = golden("recon_fused")
    runs = []
    for fuse in (False, True):
        qnn = build_qnn(Q, {})
        block = qnn.model[3]
        load_block(Q, g, block)
        block.cached_inp_features = [dev(g["cached_inp"])]
        block.cached_out_features = [dev(g["cached_out"])]
        seen = []
        orig_keep = LRF.FusedScaleLossFunction.bookkeep

        def bookkeep(self, rec):
            seen.append(float(rec.item()))
            return orig_keep(self, rec)

        LRF.FusedScaleLossFunction.bookkeep, prev = bookkeep, LRF.FUSE_TAIL
        LRF.FUSE_TAIL = fuse
        try:
            torch.manual_seed(1005)
            res = LRF.block_recon_fused_shiftedScale(block, 12, (0.01, 0.1), qnn, None, verbose=False,
                                                     graph=graph, bias_cal=True)
        finally:
            LRF.FusedScaleLossFunction.bookkeep, LRF.FUSE_TAIL = orig_keep, prev
        out = {"rec": np.array(seen), "final": np.array(res)}
        for n in ("conv1", "conv2", "downsample"):
            m = getattr(block, n)
            out[n + "_alpha"] = m.weight_quantizer.alpha.detach().cpu().numpy()
            out[n + "_gamma"] = m.alpha_out.detach().cpu().numpy()
            out[n + "_phi"] = m.beta_out.detach().cpu().numpy()
        runs.append(out)
    for k in runs[0]:
        if k in ("rec", "final"):
            np.testing.assert_allclose(runs[1][k], runs[0][k], rtol=1e-6, err_msg=k)
        else:
            np.testing.assert_array_equal(runs[1][k], runs[0][k], err_msg=k)
    assert any(np.any(runs[1][n + "_gamma"] != 1.0) for n in ("conv1", "conv2", "downsample"))
