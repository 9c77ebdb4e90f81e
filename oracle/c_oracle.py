"""ctypes loader for the plain-C oracle (oracle/c/ssq_oracle.c).  TEST INFRASTRUCTURE
ONLY: tests/ and bench.py's cpu_baseline leg use it as a checker / CPU port."""
import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "_build", "libssq_oracle.so")
_lib = None


def build():
    subprocess.run(["make", "-s", "-C", os.path.join(HERE, "c")], check=True)
    return LIB


def load():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        lib = C.CDLL(LIB)
        P, I64, I, F = C.c_void_p, C.c_int64, C.c_int, C.c_float
        lib.ssqo_fake_quant.argtypes = [P, P, P, P, P, I64, I64, I64, F, I, I]
        lib.ssqo_init_max.argtypes = [P, I64, I64, I, I, P, P, P]
        lib.ssqo_init_mse.argtypes = [P, I64, I64, I, I, P, P, P]
        _lib = lib
    return _lib


def _p(a):
    return C.c_void_p(a.ctypes.data) if a is not None else None


def fake_quant(x, delta, zp, n_bits, sym=False, scale=1.0, codes=False, nch=None):
    x = np.ascontiguousarray(x, np.float32)
    delta = np.ascontiguousarray(np.reshape(delta, -1), np.float32)
    zp = np.ascontiguousarray(np.reshape(zp, -1), np.float32)
    nch = delta.size if nch is None else nch
    inner = 1 if nch == 1 else x.size // nch
    y = np.empty_like(x)
    c = np.empty(x.shape, np.uint8) if codes else None
    n = 2 ** n_bits
    lo, hi = (-(n // 2), n // 2 - 1) if sym else (0, n - 1)
    load().ssqo_fake_quant(_p(x), _p(y), _p(c), _p(delta), _p(zp), x.size, inner, nch, scale, lo, hi)
    return y, c


def init_scale(x, n_bits, sym=False, channel_wise=True, method="max"):
    x = np.ascontiguousarray(x, np.float32)
    rows = x.shape[0] if channel_wise else 1
    d, z, r = (np.empty(rows, np.float32) for _ in range(3))
    fn = load().ssqo_init_max if method == "max" else load().ssqo_init_mse
    fn(_p(x), rows, x.size // rows, n_bits, int(sym), _p(d), _p(z), _p(r))
    return d, z, r
