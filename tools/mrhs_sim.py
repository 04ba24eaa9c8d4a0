"""How many H^-1 sweep pairs the Riccati kernel's dual active set needs when
every sweep pair also computes s = H^-1 n_q for the next most violated
constraints (MRHS), from the exact solver's own selection order.

Builds a copy of oracle/hmpc_port.c (test infrastructure) in a temp dir with
one change -- at every selection it logs the chosen constraint and the eight
most violated ones -- and replays instances through it.  A selection is a hit
when its s was computed earlier (as the choice or as a candidate of an earlier
sweep pair); sweeps/instance counts the misses.

    python tools/mrhs_sim.py
"""
import ctypes
import os
import subprocess
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'hopper-mpc-inertial_amd'))
sys.path.insert(0, ROOT)
import hmpc_plan  # noqa: E402
from oracle import port  # noqa: E402

OLD = '''      if (sc < best) { best = sc; p = i; }
    }
    if (p < 0) break;'''
NEW = '''      if (sc < best) { best = sc; p = i; }
      if (sc < -TOL) {
        for (int a = 0; a < 8; ++a) {
          if (tk[a] < 0 || sc < tv[a]) {
            for (int b2 = 7; b2 > a; --b2) { tk[b2] = tk[b2 - 1]; tv[b2] = tv[b2 - 1]; }
            tk[a] = i; tv[a] = sc; break;
          }
        }
      }
    }
    if (g_log && g_nlog < 4000) { int* e = g_log + 9 * g_nlog++; e[0] = p; for (int a = 0; a < 8; ++a) e[1 + a] = tk[a]; }
    if (p < 0) break;'''


def build(tmp):
    src = open(os.path.join(ROOT, 'oracle', 'hmpc_port.c')).read()
    assert OLD in src
    src = src.replace(OLD, NEW).replace('    double best = -TOL;\n', '    double best = -TOL;\n    int tk[8] = {-1, -1, -1, -1, -1, -1, -1, -1}; double tv[8] = {0};\n', 1)
    src = src.replace('static int gi_solve(', 'int* g_log = 0; int g_nlog = 0;\nstatic int gi_solve(', 1)
    c = os.path.join(tmp, 'port_log.c')
    so = os.path.join(tmp, 'libport_log.so')
    open(c, 'w').write(src)
    subprocess.check_call(['gcc', '-O2', '-fPIC', '-shared', '-std=c99', '-o', so, c, '-lm'])
    return so


def main():
    with tempfile.TemporaryDirectory() as tmp:
        lib = ctypes.CDLL(build(tmp))
        VP = ctypes.c_void_p
        lib.hport_solve_batch.restype = ctypes.c_long
        lib.hport_solve_batch.argtypes = ([ctypes.c_int, ctypes.c_int] + [ctypes.c_double] * 4 +
                                          [VP, VP, ctypes.c_int, ctypes.c_long] + [VP] * 11 + [ctypes.c_int])
        port._lib = lib
        buf = (ctypes.c_int * 40000)()
        glog = ctypes.c_void_p.in_dll(lib, 'g_log')
        gn = ctypes.c_int.in_dll(lib, 'g_nlog')
        for N, B, curve, sweep in ((20, 300, False, True), (60, 100, False, False), (10, 500, True, False)):
            inst = hmpc_plan.sample_instances(B, N, curve=curve, seed=2024, mu_sweep=(0.3, 1.2) if sweep else None)
            nsel, miss = 0, {k: 0 for k in (1, 2, 3, 4, 6, 8)}
            for b in range(B):
                glog.value = ctypes.addressof(buf)
                gn.value = 0
                port.solve_batch('3f', N, *[inst[k][b:b + 1] for k in ('x_in', 'x_lin', 'x_ref', 'pf', 'C')],
                                 mu=inst['mu'][b:b + 1])
                log = np.frombuffer(buf, dtype=np.int32, count=9 * gn.value).reshape(-1, 9)
                sels = [e for e in log if e[0] >= 0]
                nsel += len(sels)
                for k in miss:
                    cache = set()
                    for e in sels:
                        if e[0] not in cache:
                            miss[k] += 1
                            cache.update(int(q) for q in e[1:1 + k] if q >= 0)
                        cache.add(int(e[0]))
            print(f'N={N} B={B}: {nsel / B:.2f} selections/instance; sweep pairs/instance with K right-hand '
                  f'sides per pair: ' + ', '.join(f'K={k} {miss[k] / B:.2f}' for k in miss))


if __name__ == '__main__':
    main()
