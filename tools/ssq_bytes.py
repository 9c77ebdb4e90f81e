"""Algorithmic HBM bytes of one ssq entry point call, from its C-ABI arguments (include/ssq.h):
every operand tensor read once and every output written once, at 4 B per fp32 element
(SURVEY §8(d)'s per-unit figures; tools/recon_roofline.py prices ResNet-18's loops with the
same figures).  Used by tools/recon_configs_trace.py through _capi.CALL_HOOK, which sees each
call's ctypes arguments; per-element scalars (delta, bias, batch indices) are negligible and
not counted.  Conv-side entry points (weight gradients, depthwise convs, im2col operands) are
outside the ssq set, as their kernels are in the trace.

    bytes_of(name, args) -> int, or None for an entry point outside the ssq set."""


def _null(a):
    return a is None or getattr(a, "value", 0) is None


def _multi_elems(n, co, ci, k):
    return [int(co[s]) * int(ci[s]) * int(k[s]) for s in range(n)]


def bytes_of(name, a):
    if name in ("ssq_gather_rows2", "ssq_gather_rows2_staged"):
        # (src0, dst0, row0, src1, dst1, row1, idx|slot, nidx, ...): rows in and out
        row = int(a[2]) + (0 if _null(a[3]) else int(a[5]))
        return 8 * int(a[7]) * row
    if name == "ssq_adaround_fwd_multi":
        # (n, W, beta, delta, dpc, zp, scale, Co, Ci, K, hard, qmin, qmax, What): W, V in, W^ out
        return 12 * sum(_multi_elems(a[0], a[7], a[8], a[9]))
    if name == "ssq_adaround_bwd_multi":
        # (n, gWhat, W, beta, delta, dpc, zp, scale, Co, Ci, K, ..., gbeta): gW^, W, V in, gV out
        return 16 * sum(_multi_elems(a[0], a[8], a[9], a[10]))
    if name == "ssq_adashift_fwd_prepared_multi":
        # (n, fpack, hterm, alpha, delta, zp, Co, Ci, K, ...): packed floors + h(beta) in, W^ out
        return 12 * sum(_multi_elems(a[0], a[6], a[7], a[8]))
    if name == "ssq_adashift_bwd_prepared_multi":
        # (n, gWhat, fpack, hterm, alpha, delta, zp, Co, Ci, K, ...): gW^ + floors + h(beta) in
        return 12 * sum(_multi_elems(a[0], a[7], a[8], a[9]))
    if name in ("ssq_epilogue_fwd", "ssq_epilogue_fwd_rows"):
        rows = name.endswith("_rows")
        # (y, [y_rows,] bias, gamma, phi, res, [res_rows,] out, yq, n, ...)
        res, out, yq, n = (a[5], a[7], a[8], a[9]) if rows else (a[4], a[5], a[6], a[7])
        n = int(n)
        return 4 * n * (1 + (not _null(res)) + (not _null(out)) + (not _null(yq)))
    if name in ("ssq_epilogue_bwd", "ssq_epilogue_bwd_rows"):
        rows = name.endswith("_rows")
        # (g, y, [y_rows,] bias, gamma, phi, res, [res_rows,] N, C, hw, relu, delta, zp, qmin,
        #  qmax, gy, gres, ...)
        if rows:
            res, N, C, hw, gy, gres = a[6], a[8], a[9], a[10], a[16], a[17]
        else:
            res, N, C, hw, gy, gres = a[5], a[6], a[7], a[8], a[14], a[15]
        n = int(N) * int(C) * int(hw)
        return 4 * n * (2 + (not _null(res)) + (not _null(gy)) + (not _null(gres)))
    if name in ("ssq_epilogue_loss_bwd", "ssq_epilogue_loss_bwd_rows"):
        rows = name.endswith("_rows")
        # (tgt_cache, idx, M, p, loss_out, y, [y_rows,] bias, gamma, phi, res, [res_rows,]
        #  res_bias, res_gamma, res_phi, N, C, hw, relu, delta, zp, qmin, qmax, gy, gres, ...)
        if rows:
            res, N, C, hw, gy, gres = a[10], a[15], a[16], a[17], a[23], a[24]
        else:
            res, N, C, hw, gy, gres = a[9], a[13], a[14], a[15], a[21], a[22]
        n = int(N) * int(C) * int(hw)
        # target rows and y in, [res in], gy [, gres] out
        return 4 * n * (2 + (not _null(res)) + (not _null(gy)) + (not _null(gres)))
    if name in ("ssq_relu_bwd", "ssq_relu6_bwd"):
        return 12 * int(a[3])
    if name in ("ssq_fq_bwd", "ssq_fq_round_bwd"):
        # (x, gy, delta, zp, n, inner, nch, qmin, qmax, gx, ...)
        return 4 * int(a[4]) * (2 + (not _null(a[9])))
    if name in ("ssq_fq_relu_bwd", "ssq_fq_relu6_bwd"):
        # (x, gy, delta, zp, n, qmin, qmax, gx, ...)
        return 4 * int(a[4]) * (2 + (not _null(a[7])))
    if name in ("ssq_fq_fwd", "ssq_fq_round_fwd"):
        # (x, y, codes, delta, zp, n, ...)
        return 8 * int(a[5]) + (0 if _null(a[2]) else int(a[5]))
    if name == "ssq_lp_loss":
        # (pred, tgt, n, M, p, loss_out, grad, ...)
        return 4 * int(a[2]) * (2 + (not _null(a[6])))
    if name == "ssq_lp_loss_rows":
        # (pred, tgt_cache, idx, row, n, M, p, loss_out, grad, ...)
        return 4 * int(a[4]) * (2 + (not _null(a[8])))
    if name in ("ssq_adam", "ssq_adam_arm"):
        # (n, p, [g,] m, v, nelem, ...): p, g, m, v in; p, m, v out
        cnt = a[5] if name == "ssq_adam" else a[4]
        return 28 * sum(int(cnt[s]) for s in range(int(a[0])))
    if name in ("ssq_bias_act", "ssq_bias_act_fq"):
        # (y, bias, res, out, [yq,] n, ...)
        if name == "ssq_bias_act":
            return 4 * int(a[4]) * (2 + (not _null(a[2])))
        return 4 * int(a[5]) * (1 + (not _null(a[2])) + (not _null(a[3])) + (not _null(a[4])))
    return None


# kernels of the trace outside the ssq set (conv arithmetic: K17 / K18 / im2col operands)
CONV_SIDE = ("wgrad", "dw_kernel", "gemm_col_epi", "maxpool")


def ssq_kernel(name):
    """True for a launch of the ssq set (an ssq:: kernel that is not conv arithmetic)."""
    return "ssq::" in name and not any(c in name for c in CONV_SIDE)
