"""ctypes binding of libssq.so (include/ssq.h) plus tensor helpers.

This is the ONLY way the Python host layer reaches the HIP kernels.  There is no CPU
fallback: if the library is missing, or a tensor is not on the HIP device, the call
raises.  torch is imported before the library is loaded so that libssq.so binds to the
HIP runtime already mapped by PyTorch (same soname, one runtime per process).
"""
import ctypes as C
import os

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("SSQ_LIB", os.path.join(_HERE, "libssq.so"))

_p = C.c_void_p
_i64 = C.c_int64
_i = C.c_int
_f = C.c_float
_sz = C.c_size_t

# name -> (restype, argtypes)
SIGNATURES = {
    "ssq_last_error": (C.c_char_p, []),
    "ssq_version": (_i, []),
    "ssq_set_variant": (_i, [_i]),
    "ssq_fq_fwd": (_i, [_p, _p, _p, _p, _p, _i64, _i64, _i64, _f, _i, _i, _p]),
    "ssq_fq_round_fwd": (_i, [_p, _p, _p, _p, _p, _i64, _i64, _i64, _f, _i, _i, _p]),
    "ssq_fq_fwd_multi": (_i, [_i, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p]),
    "ssq_fq_bwd_workspace_size": (_sz, [_i64, _i64, _i64]),
    "ssq_fq_bwd": (_i, [_p, _p, _p, _p, _i64, _i64, _i64, _i, _i, _p, _p, _p, _p, _sz, _p]),
    "ssq_fq_round_bwd": (_i, [_p, _p, _p, _p, _i64, _i64, _i64, _i, _i, _p, _p, _p, _sz, _p]),
    "ssq_fq_relu_bwd": (_i, [_p, _p, _p, _p, _i64, _i, _i, _p, _p, _p, _p, _sz, _p]),
    "ssq_fq_relu6_bwd": (_i, [_p, _p, _p, _p, _i64, _i, _i, _p, _p, _p, _p, _sz, _p]),
    "ssq_scale_init_workspace_size": (_sz, [_i64, _i64, _i]),
    "ssq_scale_init": (_i, [_p, _i64, _i64, _i, _i, _i, _i, _p, _p, _p, _p, _p, _sz, _p]),
    "ssq_shift_init_workspace_size": (_sz, [_i64, _i64, _i64, _i, _i]),
    "ssq_shift_init": (_i, [_p, _p, _p, _p, _i, _i64, _i64, _i64, _i, _i, _i, _i, _p, _p, _p, _p,
                            _sz, _p]),
    "ssq_rect_init": (_i, [_p, _p, _i, _i64, _i64, _i64, _p, _p]),
    "ssq_get_delta": (_i, [_p, _p, _p, _i, _i64, _i64, _i, _p, _p]),
    "ssq_adashift_fwd": (_i, [_p, _p, _p, _p, _p, _p, _i, _i64, _i64, _i64, _i, _i, _i, _i, _i,
                              _p, _p, _p]),
    "ssq_adashift_bwd_workspace_size": (_sz, [_i64, _i64, _i64, _i, _i]),
    "ssq_adashift_prepare": (_i, [_p, _p, _p, _p, _i, _i64, _i64, _i64, _i, _p, _p, _p, _p]),
    "ssq_adashift_fwd_prepared": (_i, [_p, _p, _p, _p, _p, _i, _i64, _i64, _i64, _i, _i, _i, _p,
                                       _p]),
    "ssq_adashift_fwd_prepared_multi": (_i, [_i] + [_p] * 10 + [_i, _i, _p, _p]),
    "ssq_adashift_bwd_prepared_workspace_size": (_sz, [_i64, _i64, _i64, _i]),
    "ssq_adashift_bwd_prepared": (_i, [_p, _p, _p, _p, _p, _p, _i, _i64, _i64, _i64, _i, _i, _f,
                                       _f, _p, _p, _p, _p, _sz, _p]),
    "ssq_adashift_bwd_prepared_multi_workspace_size": (_sz, [_i, _p, _p, _p, _i]),
    "ssq_adashift_bwd_prepared_multi": (_i, [_i] + [_p] * 11 + [_i, _f, _f, _p, _p, _p, _p, _sz,
                                                                 _p]),
    "ssq_adashift_bwd": (_i, [_p, _p, _p, _p, _p, _p, _p, _i, _i64, _i64, _i64, _i, _i, _i, _i,
                              _f, _f, _p, _p, _p, _p, _p, _sz, _p]),
    "ssq_shift_reg": (_i, [_p, _i, _i64, _i, _f, _f, _p, _p, _p]),
    "ssq_lhs_fwd": (_i, [_p, _p, _p, _p, _p, _i, _i64, _i64, _i64, _i, _i, _i, _i, _p, _p]),
    "ssq_lhs_bwd": (_i, [_p, _p, _p, _p, _p, _p, _i, _i64, _i64, _i64, _i, _i, _i, _p, _p, _sz,
                         _p]),
    "ssq_adaround_fwd": (_i, [_p, _p, _p, _i, _p, _f, _i64, _i64, _i64, _i, _i, _i, _p, _p, _p]),
    "ssq_adaround_bwd": (_i, [_p, _p, _p, _p, _i, _p, _f, _i64, _i64, _i64, _i, _i, _f, _f, _p,
                              _p, _p]),
    "ssq_adaround_fwd_multi": (_i, [_i, _p, _p, _p, _p, _p, _p, _p, _p, _p, _i, _p, _p, _p, _p]),
    "ssq_adaround_bwd_multi": (_i, [_i, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _f, _f,
                                    _p, _p, _p]),
    "ssq_round_reg_workspace_size": (_sz, [_i64]),
    "ssq_round_reg": (_i, [_p, _i64, _f, _f, _p, _p, _p, _sz, _p]),
    "ssq_inpscale_search": (_i, [_p, _p, _p, _i64, _i64, _i, _i, _f, _p, _p]),
    "ssq_inpscale_fwd": (_i, [_p, _p, _p, _p, _i64, _i64, _i, _p, _p]),
    "ssq_lp_loss_workspace_size": (_sz, [_i64]),
    "ssq_lp_loss": (_i, [_p, _p, _i64, _i64, _f, _p, _p, _p, _i, _p, _sz, _p]),
    "ssq_lp_loss_rows": (_i, [_p, _p, _p, _i64, _i64, _i64, _f, _p, _p, _p, _i, _p, _sz, _p]),
    "ssq_gather_rows2": (_i, [_p, _p, _i64, _p, _p, _i64, _p, _i64, _p]),
    "ssq_gemm_col_epilogue": (_i, [_p, _p, _p, _p, _i, _p, _p, _i, _i] + [_i64] * 8 + [_p, _p]),
    "ssq_fc_recon_workspace_size": (_sz, [_i64, _i64, _i64]),
    "ssq_fc_recon_iter": (_i, [_p, _p, _p, _i64, _p, _p, _p, _p, _p, _i, _i, _p, _i64, _i64, _f, _f,
                               _f, _f, _p, _p, _p, _p, _p, _p, _sz, _p]),
    "ssq_gather_rows2_staged": (_i, [_p, _p, _i64, _p, _p, _i64, _p, _i64, _p, _i64, _p]),
    "ssq_bias_act": (_i, [_p, _p, _p, _p, _i64, _i64, _i64, _i, _p]),
    "ssq_relu_bwd": (_i, [_p, _p, _p, _i64, _p]),
    "ssq_relu6_bwd": (_i, [_p, _p, _p, _i64, _p]),
    "ssq_bias_act_fq": (_i, [_p, _p, _p, _p, _p, _i64, _i64, _i64, _i, _p, _p, _i, _i, _p]),
    "ssq_epilogue_fwd": (_i, [_p, _p, _p, _p, _p, _p, _p, _i64, _i64, _i64, _i, _p, _p, _i, _i,
                              _p]),
    "ssq_epilogue_bwd_workspace_size": (_sz, [_i64]),
    "ssq_epilogue_bwd": (_i, [_p, _p, _p, _p, _p, _p, _i64, _i64, _i64, _i, _p, _p, _i, _i, _p,
                              _p, _p, _p, _p, _p, _p, _sz, _p]),
    "ssq_epilogue_loss_bwd": (_i, [_p, _p, _i64, _f, _p, _p, _p, _p, _p, _p, _p, _p, _p, _i64,
                                   _i64, _i64, _i, _p, _p, _i, _i, _p, _p, _p, _p, _p, _p, _p,
                                   _p, _p, _sz, _p]),
    "ssq_epilogue_fwd_rows": (_i, [_p, _p, _p, _p, _p, _p, _p, _p, _p, _i64, _i64, _i64, _i, _p,
                                   _p, _i, _i, _p, _p, _i64, _p]),
    "ssq_epilogue_bwd_rows": (_i, [_p, _p, _p, _p, _p, _p, _p, _p, _i64, _i64, _i64, _i, _p, _p,
                                   _i, _i, _p, _p, _p, _p, _p, _p, _p, _sz, _p]),
    "ssq_epilogue_loss_bwd_rows": (_i, [_p, _p, _i64, _f, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p,
                                        _p, _i64, _i64, _i64, _i, _p, _p, _i, _i, _p, _p, _p, _p,
                                        _p, _p, _p, _p, _p, _sz, _p]),
    "ssq_adam": (_i, [_i, _p, _p, _p, _p, _p, _f, _f, _f, _f, _p, _f, _f, _p]),
    "ssq_adam_arm": (_i, [_i, _p, _p, _p, _p, _f, _f, _f, _f, _p, _p]),
    "ssq_adam_take": (_i, [_p]),
    "ssq_set_deferred_finalize": (_i, [_i]),
    "ssq_flush_finalize": (_i, [_p]),
    "ssq_set_deferred_prep_fwd": (_i, [_i]),
    "ssq_set_deferred_fq_multi": (_i, [_i]),
    "ssq_flush_fq_multi": (_i, [_p]),
    "ssq_flush_prep_fwd": (_i, [_p]),
    "ssq_conv_wgrad_set_form": (_i, [_i]),
    "ssq_conv_wgrad_kind": (_i, [_i64] * 10),
    "ssq_conv_wgrad_workspace_size": (_sz, [_i64] * 10),
    "ssq_conv_wgrad": (_i, [_p, _p] + [_i64] * 10 + [_p, _p, _sz, _p]),
    "ssq_wgrad_gemm_operands": (_i, [_p, _p] + [_i64] * 9 + [_p, _p, _p]),
    "ssq_maxpool2d_fwd": (_i, [_p, _p] + [_i64] * 7 + [_p]),
    "ssq_dwconv_supported": (_i, [_i64] * 8),
    "ssq_dwconv_fwd": (_i, [_p, _p, _p] + [_i64] * 8 + [_p]),
    "ssq_dwconv_bwd_data": (_i, [_p, _p, _p] + [_i64] * 8 + [_p]),
    "ssq_pack_bits": (_i, [_i]),
    "ssq_pack_bytes": (_sz, [_i64, _i]),
    "ssq_pack_encode": (_i, [_p, _p, _p, _i, _p, _i64, _i64, _i64, _i, _i, _i, _p, _p, _p]),
    "ssq_pack_decode": (_i, [_p, _p, _p, _i, _p, _i64, _i64, _i64, _i, _i, _p, _p]),
    "ssq_stream_copy": (_i, [_p, _p, _i64, _p]),
    "ssq_stream_probe": (_i, [_p, _p, _i64, _i, _p]),
}

_lib = None


class SSQError(RuntimeError):
    pass


def load():
    """Load libssq.so once; raise loudly if it is missing (no fallback path exists)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise SSQError(f"libssq.so not found at {LIB_PATH}; build it with "
                       "`python -m shiftedscalequantization_amd.build` (hipcc, gfx950)")
    lib = C.CDLL(LIB_PATH)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


# tools (tools/recon_configs_trace.py): when set, CALL_HOOK(name, args) sees every entry
# point call before it is made (the per-iteration ledger of algorithmic bytes)
CALL_HOOK = None


def call(name, *args):
    lib = load()
    if CALL_HOOK is not None:
        CALL_HOOK(name, args)
    rc = getattr(lib, name)(*args)
    if rc != 0:
        msg = lib.ssq_last_error().decode(errors="replace")
        raise SSQError(f"{name} failed (rc={rc}): {msg}")


def query(name, *args):
    return getattr(load(), name)(*args)


# ------------------------------------------------------------------ tensor helpers
def check(t, name="tensor"):
    """Kernels run on the HIP device only (no CPU fallback)."""
    if not isinstance(t, torch.Tensor):
        raise TypeError(f"{name}: expected a torch.Tensor")
    if t.device.type != "cuda":
        raise SSQError(f"{name}: ssq kernels run on the MI355X (HIP) device only; got {t.device}")
    if t.dtype != torch.float32:
        raise SSQError(f"{name}: expected float32, got {t.dtype}")
    return t


def ptr(t):
    return None if t is None else C.c_void_p(t.data_ptr())


# In-place row views (kernels.rows_view): data_ptr of a batch buffer -> (buffer, cache, idx)
# while the buffer stands for cache[idx] without having been gathered.
ROW_VIEWS = {}


# A pending stage of a chunk-replayed iteration's device words: (ring row, static slot).  The
# iteration's first K13 row-view forward performs it (ssq_epilogue_fwd_rows stage_*) and
# reads its row maps from the ring row; any other kernel call first performs it as a copy.
ROW_STAGE = []


def flush_row_stage():
    if ROW_STAGE:
        src, dst = ROW_STAGE.pop()
        dst.copy_(src)


def take_row_stage():
    """(ring row, static slot) of the pending stage, now the caller's to perform, or None."""
    return ROW_STAGE.pop() if ROW_STAGE else None


def materialize_rows(t):
    """Gather a registered row view into its buffer (one ssq_gather_rows2) and unregister it;
    a no-op for any other tensor."""
    flush_row_stage()
    e = ROW_VIEWS.pop(t.data_ptr(), None)
    if e is not None:
        buf, cache, idx = e
        call("ssq_gather_rows2", ptr(cache), ptr(buf), cache[0].numel(), None, None, 0, ptr(idx),
             idx.numel(), stream_of(buf))


def fptr(t, name="tensor"):
    """Device pointer of a contiguous fp32 tensor (made contiguous if needed).  A row view
    is gathered first: a kernel that does not read the rows in place sees the batch."""
    if t is None:
        return None, None
    check(t, name)
    if ROW_STAGE:
        flush_row_stage()
    if ROW_VIEWS:
        materialize_rows(t)
    t = t.contiguous()
    return t, C.c_void_p(t.data_ptr())


def stream_of(t):
    return C.c_void_p(torch.cuda.current_stream(t.device).cuda_stream)


_ws_cache = {}


_ws_scope = None


class workspace_scope:
    """Route workspace() to a private cache, e.g. for one captured HIP graph: the buffers
    allocated during capture belong to that graph and must never be resized under it."""

    def __init__(self, cache=None):
        self.cache = {} if cache is None else cache

    def __enter__(self):
        global _ws_scope
        self.prev, _ws_scope = _ws_scope, self.cache
        return self.cache

    def __exit__(self, *exc):
        global _ws_scope
        _ws_scope = self.prev


def workspace(nbytes, device, slot=None):
    """Per-(device, stream, slot) scratch buffer for kernel partials (grown, never shrunk).
    `slot` names a buffer that only its producer writes (the deferred finalizes read their
    partials after other launches have run: include/ssq.h)."""
    if nbytes == 0:
        return None, 0
    cache = _ws_cache if _ws_scope is None else _ws_scope
    key = (device.index, torch.cuda.current_stream(device).cuda_stream, slot)
    buf = cache.get(key)
    if buf is None or buf.numel() < nbytes:
        buf = torch.empty(max(int(nbytes), 1 << 16), dtype=torch.uint8, device=device)
        cache[key] = buf
    return C.c_void_p(buf.data_ptr()), buf.numel()


def shifts_arg(shifts):
    arr = (C.c_float * len(shifts))(*[float(s) for s in shifts])
    return arr
