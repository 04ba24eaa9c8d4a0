"""The C-ABI library loads and exports every entry point include/hmpc.h
declares (no compute without a GPU)."""
import ctypes
import os
import re

import pytest

import hmpc

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    src = open(os.path.join(ROOT, 'include', 'hmpc.h')).read()
    src = re.sub(r'/\*.*?\*/', '', src, flags=re.S)
    return sorted(set(re.findall(r'\b(hmpc_[a-z_]+)\s*\(', src)))


def test_header_declares_the_boundary():
    syms = declared_symbols()
    for s in ('hmpc_create', 'hmpc_destroy', 'hmpc_solve_batch', 'hmpc_solve_batch_host',
              'hmpc_mpcontrol_batch'):
        assert s in syms


def test_library_exports_every_declared_symbol():
    lib = ctypes.CDLL(hmpc.LIB_PATH)
    for s in declared_symbols():
        assert hasattr(lib, s), s
    # and the ctypes signature table covers exactly the header
    assert sorted(hmpc.SIGNATURES) == declared_symbols()


def test_version_and_horizons():
    lib = hmpc.load()
    assert lib.hmpc_version() == 10502   # 1.5.2: completion event at a stream switch; 1.5.1: N = 60 names the last solve's kernel; 1.5: + hmpc_overflow_total; 1.4: + hmpc_set_order (1.3: stats, refinement; 1.2: planner, CasADi, precisions 4-5, capacity)
    hs = hmpc.supported_horizons('3f')
    assert 10 in hs and 20 in hs
    assert hmpc.supported_horizons('2f') == hs


def test_argument_errors_do_not_need_a_gpu():
    lib = hmpc.load()
    h = ctypes.c_void_p()
    J = (ctypes.c_double * 9)(*([1.0] * 9))
    r = (ctypes.c_double * 3)(0, 0, 0)
    assert lib.hmpc_create(ctypes.byref(h), 7, 10, 0.02, 7.5, 9.807, 1.0, J, r, 0, 0) == -1
    assert lib.hmpc_create(ctypes.byref(h), 3, 10, -1.0, 7.5, 9.807, 1.0, J, r, 0, 0) == -1
    # horizons without a dedicated kernel run on the generic one up to N = 128
    assert lib.hmpc_create(ctypes.byref(h), 3, 129, 0.02, 7.5, 9.807, 1.0, J, r, 0, 0) == -2
    assert lib.hmpc_destroy(None) == -1
    assert lib.hmpc_set_precision(None, 1) == -1
    assert lib.hmpc_set_order(None, 0) == -1
    assert lib.hmpc_set_refinement(None, 2) == -1


def test_missing_library_fails_loudly(tmp_path):
    with pytest.raises(RuntimeError, match='no CPU fallback'):
        hmpc.load(str(tmp_path / 'nope.so'))
