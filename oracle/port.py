"""TEST INFRASTRUCTURE ONLY -- ctypes binding of oracle/libhmpc_port.so, the C
restatement of the reference's QP (oracle/hmpc_port.c).  Used by tests/ as a
second checker and by bench.py as the multi-core CPU baseline ("port")."""
from __future__ import annotations

import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, 'libhmpc_port.so')
_lib = None


def load():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f'{LIB_PATH} missing: run `make -C oracle`')
        lib = ctypes.CDLL(LIB_PATH)
        VP = ctypes.c_void_p
        lib.hport_solve_batch.restype = ctypes.c_long
        lib.hport_solve_batch.argtypes = ([ctypes.c_int, ctypes.c_int] + [ctypes.c_double] * 4 +
                                          [VP, VP, ctypes.c_int, ctypes.c_long] + [VP] * 11 +
                                          [ctypes.c_int])
        _lib = lib
    return _lib


def solve_batch(variant, N, x_in, x_lin, x_ref, pf, C, mu=None, uref_mode='aliased', nthreads=1,
                t=0.02, m=7.5, g=9.807, mu_default=1.0, Jinv=None, rh=None):
    """Exact solves of B instances (same layout as include/hmpc.h)."""
    from . import hmpc_oracle as ho
    lib = load()
    c = ho.runner_constants()
    Jinv = np.ascontiguousarray(c['Jinv'] if Jinv is None else Jinv, dtype=np.float64)
    rh = np.ascontiguousarray(c['rh'] if rh is None else rh, dtype=np.float64)
    f = lambda a: np.ascontiguousarray(np.asarray(a, dtype=np.float64))  # noqa: E731
    x_in, x_lin, x_ref, pf, C = f(x_in), f(x_lin), f(x_ref), f(pf), f(C)
    B = x_in.shape[0]
    mu_a = None if mu is None else f(np.broadcast_to(np.asarray(mu, dtype=np.float64), (B,)))
    u = np.zeros((B, N, 6))
    x = np.zeros((B, N + 1, 12))
    obj = np.zeros(B)
    st = np.zeros(B, dtype=np.int32)
    it = np.zeros(B, dtype=np.int32)
    p = lambda a: None if a is None else a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
    var = {'3f': 3, '2f': 2}[variant]
    lib.hport_solve_batch(var, N, t, m, g, mu_default, p(Jinv), p(rh),
                          1 if uref_mode == 'aliased' else 0, B, p(x_in), p(x_lin), p(x_ref), p(pf),
                          p(C), p(mu_a), p(u), p(x), p(obj), p(st), p(it), int(nthreads))
    return dict(u=u, x=x, obj=obj, status=st, iters=it)
