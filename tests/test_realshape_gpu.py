"""Reference-pinned parity at the REAL block shapes of BASELINE configs 2-5
(tests/golden/real_<case>.npz, made by make_golden.gen_real_shapes from the reference on
CPU; the seeded nets and inputs are rebuilt here from tests/golden/realshape.py):

  r18_layer4_0  ResNet-18 layer4.0 BasicBlock 256 -> 512 (GEMM-conv policy shapes)
  r50_layer1_0  ResNet-50 layer1.0 Bottleneck 64 -> 256
  mbv2_960      MobileNetV2 InvertedResidual with a 960-channel depthwise conv
  rgx_g9        RegNetX-3200M ResBottleneck 192 -> 432, 9-group conv, 1x1 projection

For each: block_recon_fused_shiftedScale (layer_recon_fused_shiftedScale.py:23-141) and
BRECQ's AdaRound block_reconstruction (block_recon.py:12-117), checked three ways:
  * inputs: folded weights hash-identical to the reference's, weight deltas / zero points
    and the shift rounding state beta bit-identical;
  * gradients, teacher-forced: at iterations GRAD_STEPS the loop's shift logits are set to
    the reference's values at that iteration, and the alpha gradient the loop then computes
    is compared per tensor with the reference's and with the EXACT gradient there (the
    reference's own computation in float64): within 1e-5 * max|g| of the exact one, or about
    as close to it as the reference's own fp32 gradient is (which itself misses it by up to
    ~1.7e-5 * max|g| on these goldens) -- see grad_stats; BRECQ's V gradient at iteration 0
    (V is the identical init) on fixed sampled entries, to 1e-5 of the reference's;
  * trajectory: identical batch draws, per-iteration losses to rtol 1e-5, learned
    parameters walk-bounded, hard decisions identical (hash of the hard weights) except
    near-ties, which are counted and bounded.
"""
import os
import sys

import numpy as np
import pytest
import torch
import torch.nn as nn

from conftest import assert_walk_bounded

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden"))
import realshape as RS  # noqa: E402

pytestmark = pytest.mark.gpu
SHIFTS = [31 / 32, 33 / 32, 1.0]
CASES = list(RS.CASES)
GRAD_TOL = 1e-5           # |g - g_exact| <= GRAD_TOL * max|g|, per tensor ...
TRUTH_FACTOR = 2.0        # ... or within 2x the reference's own fp32 distance to g_exact


@pytest.fixture(scope="module")
def Q():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from shiftedscalequantization_amd import quant
    return quant


def dev(a):
    return torch.as_tensor(np.asarray(a)).cuda()


def host(t):
    return t.detach().float().cpu().numpy()


def parity_report(test, **stats):
    import json
    rec = {"test": test, **{k: float(v) for k, v in stats.items()}}
    print("PARITY", json.dumps(rec))
    path = os.environ.get("SSQ_PARITY_LOG")
    if path:
        with open(path, "a") as f:
            f.write(json.dumps(rec) + "\n")


def our_block(kind, cin, cout):
    from shiftedscalequantization_amd import nets
    if kind == "basic1":
        return nets.BasicBlock(cin, cout)
    if kind == "basic":
        ds = nn.Sequential(nn.Conv2d(cin, cout, 1, stride=2, bias=False), nn.BatchNorm2d(cout))
        return nets.BasicBlock(cin, cout, stride=2, downsample=ds)
    if kind == "bottleneck":
        ds = nn.Sequential(nn.Conv2d(cin, cout, 1, stride=1, bias=False), nn.BatchNorm2d(cout))
        return nets.Bottleneck(cin, cout // 4, stride=1, downsample=ds)
    if kind == "inverted":
        return nets.InvertedResidual(cin, cout, 1, 6)
    return nets.ResBottleneckBlock(cin, cout, 2, 48)


def real_qnn(Q, case, g, cuda=True, bits_w=2, bits_a=4):
    """The seeded FP net of `case`, wrapped (BN folded on the CPU as the reference does)."""
    kind, cin, cout, _ = RS.CASES[case]
    net = RS.seed_net(RS.wrap(our_block(kind, cin, cout), cout))
    assert RS.layout(net) == [str(s) for s in g["layout"]]
    assert RS.seed_sha(net) == str(g["seed_sha"][0]), "seeded FP parameters differ"
    wq = {"n_bits": bits_w, "channel_wise": True, "scale_method": "max"}
    aq = {"n_bits": bits_a, "channel_wise": False, "scale_method": "mse", "leaf_param": True}
    qnn = Q.QuantModel(net, wq, aq).eval()
    return qnn.cuda() if cuda else qnn


def named_qms(block, Q):
    return [(n, m) for n, m in block.named_modules() if isinstance(m, Q.QuantModule)]


def init_weights(Q, case, g, stats):
    """Seeded net on the device, weight quantizers initialised ('max') by one forward; the
    folded weights, deltas and zero points checked against the reference's."""
    qnn = real_qnn(Q, case, g)
    block = qnn.model[0]
    x = RS.calib_input(case).cuda()
    qnn.set_quant_state(True, False)
    with torch.no_grad():
        qnn(x)
    qms = named_qms(block, Q)
    assert [n for n, _ in qms] == [str(s) for s in g["qms"]]
    for n, m in qms:
        assert RS.sha(host(m.org_weight)) == str(g[f"{n}_w_sha"][0]), n
        assert RS.sha(host(m.org_bias)) == str(g[f"{n}_b_sha"][0]), n
        np.testing.assert_array_equal(host(m.weight_quantizer.delta).reshape(-1), g[f"{n}_delta"])
        np.testing.assert_array_equal(host(m.weight_quantizer.zero_point).reshape(-1), g[f"{n}_zp"])
    stats["n_weights"] = sum(m.org_weight.numel() for _, m in qms)
    return qnn, block, x, qms


def setup_fused(Q, case, g, stats, cached=None):
    """`cached`: the fixture holding the reference's FP block output when `g` does not
    (the bias_cal / long-horizon fixtures: the same seeded case, checked by hash)."""
    from shiftedscalequantization_amd import drivers as D
    if cached is not None:
        assert str(cached["cached_out_sha"][0]) == str(g["cached_out_sha"][0])
        g = dict(g, cached_out=cached["cached_out"], layout=cached["layout"],
                 seed_sha=cached["seed_sha"])
    qnn, block, x, qms = init_weights(Q, case, g, stats)
    for n, m in qms:
        m.weight_quantizer = Q.ChannelQuant(1.0, uaq=m.weight_quantizer, weight_tensor=m.org_weight,
                                            shiftTarget=SHIFTS, name="." + n)
        m.use_weight_quant = True
    qnn.set_quant_state(False, False)
    with torch.no_grad():
        fp = host(block(x))
    stats["fp_out_rel_err"] = np.abs(fp - g["cached_out"]).max() / np.abs(g["cached_out"]).max()
    assert stats["fp_out_rel_err"] <= 1e-5
    # the loop reconstructs against the reference's own FP output
    block.cached_inp_features, block.cached_out_features = [x.clone()], [dev(g["cached_out"])]
    D.set_quant_state_block(qnn, [".model.0"], "", True)
    for n, m in qms:
        ref = str(g[f"{n}_beta0_sha"][0])
        if ref:
            assert RS.sha(host(m.weight_quantizer.beta)) == ref, n
    return qnn, block, qms


def run_fused(Q, qnn, block, probe_fn, iters=RS.ITERS, bias_cal=False):
    import importlib
    LRF = importlib.import_module("shiftedscalequantization_amd.quant.layer_recon_fused_shiftedScale")
    E = importlib.import_module("shiftedscalequantization_amd.quant._engine")
    seen_perms, seen_rec = [], []
    orig_draw, orig_keep = LRF.BatchFeeder.draw, LRF.FusedScaleLossFunction.bookkeep

    def draw(self):
        p = orig_draw(self)
        seen_perms.append(p.clone())
        return p

    def bookkeep(self, rec):
        seen_rec.append(float(rec.item()))     # read now: a graph replay overwrites it
        return orig_keep(self, rec)

    LRF.BatchFeeder.draw, LRF.FusedScaleLossFunction.bookkeep = draw, bookkeep
    E.ITER_PROBE[0] = probe_fn
    try:
        torch.manual_seed(1005)
        res = LRF.block_recon_fused_shiftedScale(block, iters, (0.01, 0.1), qnn, None,
                                                 verbose=False, bias_cal=bias_cal)
    finally:
        LRF.BatchFeeder.draw, LRF.FusedScaleLossFunction.bookkeep = orig_draw, orig_keep
        E.ITER_PROBE[0] = None
    return np.stack([p.numpy() for p in seen_perms]), np.array(seen_rec), np.array(res)


def grad_recorder(steps, force=None):
    """Probe: grads of iteration s are read at the start of iteration s + 1; with `force`
    (step -> list of parameter values) the parameters are overwritten at the start of
    those iterations (teacher forcing)."""
    got, before = {}, {}

    def probe(i, params):
        if i - 1 in steps:
            got[i - 1] = [host(p.grad) for p in params]
        if force is not None and i in force:
            before[i] = [host(p) for p in params]
            with torch.no_grad():
                for p, v in zip(params, force[i]):
                    p.copy_(dev(v).view(p.shape))
    return probe, got, before


def grad_stats(stats, tag, got, ref, truth=None):
    """Per tensor: err = max|g - g_ref| / max|g_ref|; with `truth` (the reference's own
    gradient evaluated in float64 at the same parameters and batch, make_golden._fused_truth)
    also our and the reference's distance to it.  Returns the worst excess over the bound:
    err_truth <= max(GRAD_TOL, TRUTH_FACTOR * ref_truth) when the truth is known (our fp32
    gradient is within 1e-5 * max|g| of the exact one, or about as close to it as the
    reference's own fp32 gradient), else err <= GRAD_TOL.  <= 1 passes."""
    worst = 0.0
    for j, (a, r) in enumerate(zip(got, ref)):
        a = np.asarray(a, np.float64)
        r = np.asarray(r, np.float64).reshape(a.shape)
        err = np.abs(a - r).max(initial=0.0) / max(np.abs(r).max(initial=0.0), 1e-30)
        stats[f"{tag}_t{j}"] = err
        if truth is None:
            worst = max(worst, err / GRAD_TOL)
            continue
        t = np.asarray(truth[j], np.float64).reshape(a.shape)
        tmax = max(np.abs(t).max(initial=0.0), 1e-30)
        e_t = np.abs(a - t).max(initial=0.0) / tmax
        r_t = np.abs(r - t).max(initial=0.0) / tmax
        stats[f"{tag}_t{j}_vs_fp64"] = e_t
        stats[f"{tag}_t{j}_ref_vs_fp64"] = r_t
        worst = max(worst, e_t / max(GRAD_TOL, TRUTH_FACTOR * r_t))
    return worst


def truths(g, prefix, s, n_p):
    key = f"{prefix}gs{s}_t0"
    return [g[f"{prefix}gs{s}_t{j}"] for j in range(n_p)] if key in g else None


@pytest.mark.parametrize("case", CASES)
def test_real_fused_gradients_teacher_forced(Q, golden, case):
    g = golden(f"real_{case}")
    stats = {}
    qnn, block, qms = setup_fused(Q, case, g, stats)
    steps = [int(s) for s in g["grad_steps"]]
    n_p = len(qms)
    force = {s: [g[f"gs{s}_p{j}"] for j in range(n_p)] for s in steps}
    probe, got, before = grad_recorder(steps, force)
    perms, rec, _ = run_fused(Q, qnn, block, probe)
    np.testing.assert_array_equal(perms, g["perms"])
    # iteration 0's alpha is our own init: the reference's to a few ulps (log-domain init)
    stats["init_dev"] = max(np.abs(before[0][j].reshape(-1) - force[0][j].reshape(-1)).max()
                            for j in range(n_p))
    worst = 0.0
    for s in steps:
        worst = max(worst, grad_stats(stats, f"g{s}", got[s], [g[f"gs{s}_g{j}"] for j in range(n_p)],
                                      truths(g, "", s, n_p)))
    stats["worst_grad_over_bound"] = worst
    parity_report(f"real_fused_grad[{case}]", **stats)
    assert stats["init_dev"] <= 5e-7
    assert worst <= 1.0, stats


def param_index(qms, bias_cal):
    """Positions of each module's (alpha, gamma^z, phi^z) in the loop's parameter list:
    alpha only, or alpha / alpha_out / beta_out per QuantModule with bias_cal (the order of
    the reference's commented opt_params lines, layer_recon_fused_shiftedScale.py:66-68)."""
    k = 3 if bias_cal else 1
    return {n: (j * k, j * k + 1, j * k + 2) if bias_cal else (j,) for j, (n, _) in enumerate(qms)}


def check_trajectory(g, qms, stats, rec, res, got, steps, iters, bias_cal, walk_rows=2,
                     tight_frac=0.95, free_tol=2e-4, aff_walk_frac=0.05, dev_max=None):
    """The free-running loop against the reference's trajectory: per-iteration and final
    losses to rtol 1e-5; shift logits alpha per input-channel row: inside Adam's step budget
    (iters * 2 * lr), at most `walk_rows` live rows per layer off by > 2e-4 (near-cancelling
    gradients: Adam walks them in +-lr steps, in the reference as here), at least
    `tight_frac` of the live rows within 1e-5; the hard shift choice identical except where
    the reference's top-two logits are within the budget of each other, and then the hard
    weights hash-identical; free-running gradients within `free_tol` of the reference's;
    with bias_cal gamma^z / phi^z inside the budget, at most `aff_walk_frac` of their entries
    off by > 2e-4; with dev_max, every live row within it."""
    from oracle import ssq_ref as R
    n_p = len(qms) * (3 if bias_cal else 1)
    stats["rec_rel_err"] = np.max(np.abs(rec - g["rec_loss"][:iters]) / np.abs(g["rec_loss"][:iters]))
    stats["final_rel_err"] = np.max(np.abs(res - g["final_losses"]) / np.abs(g["final_losses"]))
    for s in steps:
        st = {}
        grad_stats(st, "", got[s], [g[f"gs{s}_g{j}"] for j in range(n_p)])
        stats[f"free_g{s}_worst"] = max(st.values())
    budget = iters * 2e-3
    flips_total = 0
    checks = []
    idx = param_index(qms, bias_cal)
    for n, m in qms:
        q = m.weight_quantizer
        a, ar = host(q.alpha), g[f"{n}_alpha"]
        a2, r2 = a.reshape(-1, a.shape[-1]), ar.reshape(-1, ar.shape[-1])
        da = np.abs(a2 - r2)
        # input channels whose shift candidates are all identical (floor(W/(d*s_i)) equal
        # for every shift) have an analytically ZERO alpha gradient: Adam turns the
        # rounding residue there into +-lr steps, in the reference as here (a random walk
        # inside the step budget, irrelevant to W^)
        w = host(m.org_weight)
        fl = np.stack(R.shift_floors(w, g[f"{n}_delta"].reshape((-1,) + (1,) * (w.ndim - 1)), SHIFTS))
        axes = (0, 1) + tuple(range(3, fl.ndim))
        degenerate = np.all(fl == fl[:1], axis=axes).reshape(-1)
        if degenerate.size != a2.shape[0]:          # depthwise: one alpha row for the tensor
            degenerate = np.full(a2.shape[0], bool(np.all(fl == fl[:1])))
        rows = da.max(-1)
        live = ~degenerate
        off = live & (rows > 2e-4)
        stats[f"{n}_rows"], stats[f"{n}_degenerate_rows"] = a2.shape[0], int(degenerate.sum())
        stats[f"{n}_walking_rows"] = int(off.sum())
        stats[f"{n}_tight_frac"] = float(np.mean(rows[live] <= 1e-5)) if live.any() else 1.0
        stats[f"{n}_alpha_dev_median"] = float(np.median(rows[live])) if live.any() else 0.0
        stats[f"{n}_alpha_dev_max"] = float(rows.max(initial=0.0))
        checks.append((n, off, rows))
        if bias_cal:
            for key, t in (("gamma", m.alpha_out), ("phi", m.beta_out)):
                d_ = np.abs(host(t).reshape(-1) - g[f"{n}_{key}"].reshape(-1))
                stats[f"{n}_{key}_dev_max"] = float(d_.max())
                stats[f"{n}_{key}_walkers"] = int((d_ > 2e-4).sum())
                assert d_.max() <= budget, (n, key, float(d_.max()))
                assert (d_ > 2e-4).sum() <= max(1, round(aff_walk_frac * d_.size)), (n, key, stats)
        # beta: init_v_beta at the loop start, never optimised (rtol 1e-5: its log-domain
        # init runs on the device, a few ulps off the reference's CPU log)
        bi = RS.sub_idx(q.beta.numel())
        np.testing.assert_allclose(host(q.beta).reshape(-1)[bi], g[f"{n}_beta_sub"], rtol=1e-5, atol=1e-6)
        flip = (np.argmax(a2, -1) != np.argmax(r2, -1)) & ~degenerate
        srt = np.sort(r2, -1)
        gap = srt[:, -1] - srt[:, -2]
        assert np.all(gap[flip] <= budget), (n, gap[flip])
        stats[f"{n}_shift_flips"] = int(flip.sum())
        flips_total += int(flip.sum())
        with torch.no_grad():
            wh = RS.sha(host(q(m.weight)))
        if not flip.any():
            assert wh == str(g[f"{n}_what_hard_sha"][0]), f"{n}: hard weights differ"
        stats[f"{n}_hard_identical"] = float(wh == str(g[f"{n}_what_hard_sha"][0]))
    stats["shift_flips"] = flips_total
    np.testing.assert_allclose(rec, g["rec_loss"][:iters], rtol=1e-5)
    np.testing.assert_allclose(res, g["final_losses"], rtol=1e-5)
    for n, off, rows in checks:
        assert rows.max(initial=0.0) <= budget, n
        if dev_max is not None:
            assert rows.max(initial=0.0) <= dev_max, (n, rows.max())
        assert off.sum() <= walk_rows, (n, np.nonzero(off)[0], stats)
        assert stats[f"{n}_tight_frac"] >= tight_frac, (n, stats[f"{n}_tight_frac"])
    for s in steps:
        assert stats[f"free_g{s}_worst"] <= free_tol, (s, stats[f"free_g{s}_worst"])


@pytest.mark.parametrize("case", CASES)
def test_real_fused_trajectory(Q, golden, case):
    """20 iterations at the real shapes; bounds at the observed values plus a margin
    (observed r3, profiles/r3_parity_grads_realshape.jsonl: 0-2 walking rows per layer,
    tight fractions 0.958-1.0, free-running gradients <= 1.0e-4)."""
    g = golden(f"real_{case}")
    stats = {}
    qnn, block, qms = setup_fused(Q, case, g, stats)
    steps = [int(s) for s in g["grad_steps"]]
    probe, got, _ = grad_recorder(steps)
    perms, rec, res = run_fused(Q, qnn, block, probe)
    np.testing.assert_array_equal(perms, g["perms"])
    try:
        check_trajectory(g, qms, stats, rec, res, got, steps, RS.ITERS, False)
    finally:
        parity_report(f"real_fused_traj[{case}]", **stats)


BIASCAL_CASES = ["r18_layer4_0", "r18_layer1_0"]


@pytest.mark.parametrize("case", BIASCAL_CASES)
def test_real_biascal_gradients_teacher_forced(Q, golden, case):
    """--bias_cal against the reference run under the oracle-side shim that realises its
    commented opt_params lines (make_golden._BiasCalAdam): at GRAD_STEPS the loop's alpha,
    gamma^z and phi^z are set to the reference's values and the gradients it computes are
    held to the float64 truth (grad_stats), tensor by tensor."""
    g = golden(f"real_{case}_biascal")
    stats = {}
    qnn, block, qms = setup_fused(Q, case, g, stats, cached=golden(f"real_{case}"))
    steps = [int(s) for s in g["grad_steps"]]
    n_p = 3 * len(qms)
    force = {s: [g[f"gs{s}_p{j}"] for j in range(n_p)] for s in steps}
    probe, got, before = grad_recorder(steps, force)
    perms, rec, _ = run_fused(Q, qnn, block, probe, bias_cal=True)
    np.testing.assert_array_equal(perms, g["perms"])
    stats["init_dev"] = max(np.abs(before[0][j].reshape(-1) - force[0][j].reshape(-1)).max()
                            for j in range(n_p))
    worst = 0.0
    for s in steps:
        worst = max(worst, grad_stats(stats, f"g{s}", got[s], [g[f"gs{s}_g{j}"] for j in range(n_p)],
                                      truths(g, "", s, n_p)))
    stats["worst_grad_over_bound"] = worst
    parity_report(f"real_biascal_grad[{case}]", **stats)
    assert stats["init_dev"] <= 5e-7
    assert worst <= 1.0, stats


@pytest.mark.parametrize("case", BIASCAL_CASES)
def test_real_biascal_trajectory(Q, golden, case):
    g = golden(f"real_{case}_biascal")
    stats = {}
    qnn, block, qms = setup_fused(Q, case, g, stats, cached=golden(f"real_{case}"))
    steps = [int(s) for s in g["grad_steps"]]
    probe, got, _ = grad_recorder(steps)
    perms, rec, res = run_fused(Q, qnn, block, probe, bias_cal=True)
    np.testing.assert_array_equal(perms, g["perms"])
    try:
        check_trajectory(g, qms, stats, rec, res, got, steps, RS.ITERS, True)
    finally:
        parity_report(f"real_biascal_traj[{case}]", **stats)


@pytest.mark.parametrize("bias_cal", [False, True])
def test_long_horizon_gradients_teacher_forced(Q, golden, bias_cal):
    """The driver's 625-iteration horizon on the ResNet-18 layer1.0 shape (both b / b2
    schedules run to their ends): teacher-forced gradients at LONG_GRAD_STEPS against the
    float64 truth."""
    case = "r18_layer1_0"
    g = golden(f"long_{case}" + ("_biascal" if bias_cal else ""))
    stats = {}
    qnn, block, qms = setup_fused(Q, case, g, stats, cached=golden(f"real_{case}"))
    steps = [int(s) for s in g["grad_steps"]]
    n_p = len(qms) * (3 if bias_cal else 1)
    force = {s: [g[f"gs{s}_p{j}"] for j in range(n_p)] for s in steps}
    probe, got, before = grad_recorder(steps, force)
    perms, rec, _ = run_fused(Q, qnn, block, probe, iters=RS.LONG_ITERS, bias_cal=bias_cal)
    np.testing.assert_array_equal(perms, g["perms"])
    worst = 0.0
    for s in steps:
        worst = max(worst, grad_stats(stats, f"g{s}", got[s], [g[f"gs{s}_g{j}"] for j in range(n_p)],
                                      truths(g, "", s, n_p)))
    stats["worst_grad_over_bound"] = worst
    parity_report(f"long_grad[bias_cal={bias_cal}]", **stats)
    assert worst <= 1.0, stats


@pytest.mark.parametrize("bias_cal", [False, True])
def test_long_horizon_trajectory(Q, golden, bias_cal):
    """625 free-running iterations against the reference's: every iteration's loss to
    rtol 1e-5, the learned parameters and the hard decisions as check_trajectory."""
    case = "r18_layer1_0"
    g = golden(f"long_{case}" + ("_biascal" if bias_cal else ""))
    stats = {}
    qnn, block, qms = setup_fused(Q, case, g, stats, cached=golden(f"real_{case}"))
    steps = [int(s) for s in g["grad_steps"]]
    probe, got, _ = grad_recorder(steps)
    perms, rec, res = run_fused(Q, qnn, block, probe, iters=RS.LONG_ITERS, bias_cal=bias_cal)
    np.testing.assert_array_equal(perms, g["perms"])
    try:
        # 625 Adam steps accumulate a few 1e-6 per row (observed r4: max row deviation
        # 1.75e-5, no row off by > 2e-4, 94-100 % of the rows within 1e-5): every row within
        # 1e-4, at least 90 % within 1e-5
        check_trajectory(g, qms, stats, rec, res, got, steps, RS.LONG_ITERS, bias_cal,
                         walk_rows=0, tight_frac=0.9, dev_max=1e-4)
    finally:
        parity_report(f"long_traj[bias_cal={bias_cal}]", **stats)


def test_real_layer_shift_w4a8_matches_reference(Q, golden):
    """Config 1 at the real ResNet-18 layer1.0.conv1 shape (W4A8, layer_recon_shiftedScale:
    layer_recon_shiftedScale.py:262-338): the shift phase's losses, alpha trajectory and
    teacher-forced gradients (against the float64 truth), its hard weights; then the
    AdaRound phase's losses, selected deltas, beta (walk-bounded, hard rounding decided
    where the reference's beta is outside the walk budget) and hard weights."""
    import importlib
    from shiftedscalequantization_amd import drivers as D
    E = importlib.import_module("shiftedscalequantization_amd.quant._engine")
    case = "r18_layer1_0"
    g = golden(f"real_{case}_layer_shift_w4a8")
    stats = {}
    qnn = real_qnn(Q, case, g, bits_w=4, bits_a=8)
    x = RS.calib_input(case).cuda()
    qnn.set_quant_state(True, False)
    with torch.no_grad():
        qnn(x)
    m = qnn.model[0].conv1
    assert RS.sha(host(m.org_weight)) == str(g["w_sha"][0])
    assert RS.sha(host(m.org_bias)) == str(g["b_sha"][0])
    np.testing.assert_array_equal(host(m.weight_quantizer.delta).reshape(-1), g["delta"])
    np.testing.assert_array_equal(host(m.weight_quantizer.zero_point).reshape(-1), g["zp"])
    D.build_ShiftedChannelQuant(qnn, [".model.0"], "", shiftTarget=SHIFTS, skipShiftLayer=[])
    qnn.set_quant_state(False, False)
    with torch.no_grad():
        fp = host(m(x))
    stats["fp_out_rel_err"] = np.abs(fp - g["cached_out"]).max() / np.abs(g["cached_out"]).max()
    assert stats["fp_out_rel_err"] <= 1e-5
    m.cached_inp_features, m.cached_out_features = [x.clone()], [dev(g["cached_out"])]
    m.use_weight_quant = True
    q = m.weight_quantizer
    iters = int(g["iters"][0])
    steps = [int(s_) for s_ in g["shift_grad_steps"]]
    # teacher-forced at the recorded steps (alpha set to the reference's value there): the
    # gradient is held to the float64 truth, and the trajectory stays the reference's
    probe, got, before = grad_recorder(steps, {s_: [g[f"shift_gs{s_}_p0"]] for s_ in steps})
    E.ITER_PROBE[0] = probe
    try:
        torch.manual_seed(1005)
        l1 = Q.layer_recon_shiftedScale(m, iters, 0.1, qnn, None, verbose=False)
    finally:
        E.ITER_PROBE[0] = None
    stats["shift_final_rel_err"] = np.max(np.abs(np.array(l1) - g["shift_final"]) / np.abs(g["shift_final"]))
    np.testing.assert_allclose(l1, g["shift_final"], rtol=1e-5)
    assert RS.sha(np.stack([host(t) for t in q.x_q])) == str(g["shift_xq_sha"][0])
    da = np.abs(host(q.alpha) - g["shift_alpha"])
    stats["shift_alpha_dev"] = da.max()
    stats["shift_alpha_walkers"] = assert_walk_bounded(da, 1e-5, iters * 2e-3, frac=0.02,
                                                      what="shift alpha")
    worst = 0.0
    for s_ in steps:
        worst = max(worst, grad_stats(stats, f"shift_g{s_}", got[s_], [g[f"shift_gs{s_}_g0"]],
                                      truths(g, "shift_", s_, 1)))
    stats["shift_grad_worst_over_bound"] = worst
    stats["shift_init_dev"] = np.abs(before[0][0] - g["shift_gs0_p0"]).max()
    with torch.no_grad():
        wh = RS.sha(host(q(m.weight)))
    stats["shift_hard_identical"] = float(wh == str(g["shift_what_sha"][0]))
    q.hard_targets = False
    # the AdaRound phase, teacher-forced the same way: beta set to the reference's value at
    # the recorded steps, the gradient (ScaleLossFunction's lp term + the rounding term,
    # layer_recon_shiftedScale.py:297-338,414-486) held to its float64 truth
    ar_steps = [int(s_) for s_ in g["ar_grad_steps"]]
    probe, ar_got, ar_before = grad_recorder(ar_steps, {s_: [g[f"ar_gs{s_}_p0"]] for s_ in ar_steps})
    E.ITER_PROBE[0] = probe
    try:
        l2 = Q.layer_recon_shiftedScale(m, iters, 0.01, qnn, None, adaround=True, verbose=False)
    finally:
        E.ITER_PROBE[0] = None
    ar_worst = 0.0
    for s_ in ar_steps:
        ar_worst = max(ar_worst, grad_stats(stats, f"ar_g{s_}", ar_got[s_], [g[f"ar_gs{s_}_g0"]],
                                            truths(g, "ar_", s_, 1)))
    stats["ar_grad_worst_over_bound"] = ar_worst
    # beta at step 0 is init_beta of the selected deltas: forced to the reference's, so the
    # overwrite must have been (almost) a no-op
    stats["ar_init_dev"] = np.abs(ar_before[0][0].reshape(-1) - g["ar_gs0_p0"].reshape(-1)).max()
    stats["ar_final_rel_err"] = np.max(np.abs(np.array(l2) - g["ar_final"]) / np.abs(g["ar_final"]))
    d = host(q.delta)
    stats["ar_delta_flips"] = int(np.sum(d != g["ar_delta"]))
    bq = host(q.beta)
    db = np.abs(bq - g["ar_beta"])
    budget = iters * 2e-3
    stats["ar_beta_dev_max"] = db.max()
    stats["ar_beta_walk_frac"] = float(np.mean(db > 2e-4))
    decided = np.abs(g["ar_beta"]) > budget
    stats["ar_undecided_frac"] = float(np.mean(~decided))
    flip = (bq >= 0) != (g["ar_beta"] >= 0)
    stats["ar_round_flips"] = int(flip.sum())
    stats["ar_flips_max_abs_ref_beta"] = float(np.abs(g["ar_beta"][flip]).max(initial=0.0))
    with torch.no_grad():
        wh2 = RS.sha(host(q(m.weight)))
        # the reference sets its hard flag on the layer, not on the quantizer
        # (layer_recon_shiftedScale.py:322-323): the quantizer still rounds softly, so its
        # output carries beta's own bits (and the sigmoid's: torch's vectorised exp and
        # expf may differ by an ulp on some of the 36864 entries) -- reported, not asserted
        b_ours = q.beta.detach().clone()
        q.beta.copy_(dev(g["ar_beta"]).view(q.beta.shape))
        wh_ref_state = RS.sha(host(q(m.weight)))
        q.beta.copy_(b_ours)
    stats["ar_hard_identical"] = float(wh2 == str(g["ar_what_sha"][0]))
    stats["ar_what_from_ref_beta_identical"] = float(wh_ref_state == str(g["ar_what_sha"][0]))
    # the final losses: rtol 1e-5 (north_star) when no beta walked; a walked beta moves the
    # soft-rounded output, and with it the loss, by the walk's own size (observed r4: 1.5 %
    # of the entries by <= 1.1e-3 -> 2e-5 relative), which is the bound then
    rtol = 1e-5 if stats["ar_beta_walk_frac"] == 0.0 else 1e-4
    stats["ar_final_rtol_applied"] = rtol
    parity_report("real_layer_shift_w4a8[r18_layer1_0]", **stats)
    assert worst <= 1.0 and ar_worst <= 1.0, stats
    assert stats["shift_init_dev"] <= 5e-7 and stats["ar_init_dev"] <= 5e-7, stats
    assert stats["ar_delta_flips"] == 0, stats
    # beta: teacher-forced gradients at the exact-gradient bound (above); between the forced
    # steps Adam's first moves are +-lr whatever the gradient's size, so an entry whose
    # gradient is at the fp32 noise floor of the dL/dW sum takes the sign that summation
    # order gives it -- in the reference as here.  Those walk by <= 2 lr per step; the
    # rounding decision may flip only inside that budget (observed r5, teacher-forced:
    # beta within 7.9e-5, no entry walking, no flip, final loss 3.1e-7).
    assert db.max() <= budget and np.mean(db > 2e-4) <= 0.05, stats
    assert np.all(np.abs(g["ar_beta"][flip]) <= budget), stats
    np.testing.assert_allclose(l2, g["ar_final"], rtol=rtol)
    if stats["shift_alpha_walkers"] == 0:
        assert stats["shift_hard_identical"] == 1.0


@pytest.mark.parametrize("case", CASES)
def test_real_brecq_matches_reference(Q, golden, case):
    import importlib
    g = golden(f"real_{case}")
    stats = {}
    qnn, block, x, qms = init_weights(Q, case, g, stats)
    BR = importlib.import_module("shiftedscalequantization_amd.quant.block_recon")
    E = importlib.import_module("shiftedscalequantization_amd.quant._engine")
    seen = []
    orig_rec, orig_init = BR.LossFunction.record, BR.LossFunction.__init__

    def spy(self, rec, rnd, b):
        r = orig_rec(self, rec, rnd, b)
        seen.append(float(r))
        return r

    def init(self, *a, **k):
        orig_init(self, *a, **k)
        self.track_values = True

    probe, got, _ = grad_recorder(list(RS.BRECQ_GRAD_STEPS))
    BR.LossFunction.record, BR.LossFunction.__init__ = spy, init
    E.ITER_PROBE[0] = probe
    try:
        torch.manual_seed(1005)
        Q.block_reconstruction(qnn, block, x, batch_size=8, iters=RS.BRECQ_ITERS, weight=0.01,
                               asym=True, b_range=(20, 2), warmup=0.2, act_quant=False,
                               opt_mode="mse")
    finally:
        BR.LossFunction.record, BR.LossFunction.__init__ = orig_rec, orig_init
        E.ITER_PROBE[0] = None
    stats["total_rel_err"] = np.max(np.abs(np.array(seen) - g["b_total_loss"]) / np.abs(g["b_total_loss"]))
    np.testing.assert_allclose(seen, g["b_total_loss"], rtol=1e-5)
    budget = RS.BRECQ_ITERS * 2e-3
    flips_total = 0
    for j, (n, m) in enumerate(qms):
        q = m.weight_quantizer
        idx = RS.sub_idx(q.alpha.numel())
        v = host(q.alpha).reshape(-1)
        dv = np.abs(v[idx] - g[f"b_{n}_V_sub"])
        stats[f"{n}_V_dev"] = dv.max()
        stats[f"{n}_V_walkers"] = assert_walk_bounded(dv, 1e-5, budget, frac=0.01, what=n)
        # gradients: iteration 0 (V is the identical init) to GRAD_TOL, the last one
        # (free-running) reported and bounded loosely; both on the sampled entries and as
        # per-output-channel L1 norms over the whole tensor
        for s in RS.BRECQ_GRAD_STEPS:
            gg = got[s][j]
            ref_max = float(g[f"b_{n}_gs{s}_max"][0])
            err = np.abs(gg.reshape(-1)[idx] - g[f"b_{n}_gs{s}_sub"]).max() / max(ref_max, 1e-30)
            l1 = RS.row_l1(gg)
            l1_err = np.max(np.abs(l1 - g[f"b_{n}_gs{s}_rowl1"]) / np.maximum(g[f"b_{n}_gs{s}_rowl1"], 1e-30))
            stats[f"{n}_g{s}_err"], stats[f"{n}_g{s}_rowl1_rel"] = err, l1_err
            if s == 0:
                assert err <= GRAD_TOL, (n, err)
                assert l1_err <= 1e-4, (n, l1_err)
            else:
                assert err <= 1e-3, (n, s, err)
        # hard rounding decision (V >= 0): flips only inside the walk budget
        ref_pos = np.unpackbits(g[f"b_{n}_V_pos"])[:v.size].astype(bool)
        flip = (v >= 0) != ref_pos
        assert np.all(np.abs(v[flip]) <= budget), (n, v[flip])
        assert flip.mean() <= 1e-4, (n, int(flip.sum()))
        stats[f"{n}_round_flips"] = int(flip.sum())
        flips_total += int(flip.sum())
        with torch.no_grad():
            wh = RS.sha(host(q(m.weight)))
        if not flip.any():
            assert wh == str(g[f"b_{n}_what_hard_sha"][0]), f"{n}: hard weights differ"
        stats[f"{n}_hard_identical"] = float(wh == str(g[f"b_{n}_what_hard_sha"][0]))
    stats["round_flips"] = flips_total
    parity_report(f"real_brecq[{case}]", **stats)
