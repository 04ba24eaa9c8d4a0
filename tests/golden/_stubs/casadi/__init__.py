"""Recording stand-in for casadi -- used ONLY by tests/golden/make_golden.py.

casadi and qpOASES are not installed in this image (no network).  The
reference's CasADi variant (src/mpc_cas_euler_3f.py) only needs symbolic
matrices (SX.sym / SX.zeros, slicing, block assignment, +, -, *, @, .T),
horzcat / vertcat / reshape and qpsol.  This stub does that symbolic algebra
with sympy (exact expression trees; numbers as binary64 Floats) and, when the
solver is called, substitutes the parameter values and reads the QP the
reference built off the expressions:

    1/2 z'Pz + q'z + r   s.t.  lbg <= A z - b... (as g(z) = A z + g0)
                               lbx <= z <= ubx

in casadi's variable order z = [vec(x) (column-major); vec(u)].  Every call
is appended to RECORD; the solve is delegated to SOLVER (make_golden.py sets
the oracle's exact solver), since qpOASES is absent.
"""
import numpy as np
import sympy

RECORD = []
SOLVER = None


def _mat(v):
    """sympy Matrix of anything the reference hands in."""
    if isinstance(v, SX):
        return v.M
    if isinstance(v, sympy.MatrixBase):
        return v
    a = np.asarray(v, dtype=np.float64)
    if a.ndim == 0:
        return sympy.Matrix([[sympy.Float(float(a))]])
    if a.ndim == 1:
        a = a.reshape(-1, 1)
    return sympy.Matrix(a.shape[0], a.shape[1], [sympy.Float(float(x)) for x in a.ravel()])


def _wrap(m):
    return SX(m if isinstance(m, sympy.MatrixBase) else sympy.Matrix([[m]]))


class SX:
    __array_priority__ = 1000
    __array_ufunc__ = None

    def __init__(self, M):
        self.M = sympy.Matrix(M)

    @staticmethod
    def zeros(n, m=1):
        return SX(sympy.zeros(n, m))

    @staticmethod
    def sym(name, n, m=1):
        return SX(sympy.Matrix(n, m, lambda i, j: sympy.Symbol(f'{name}_{i}_{j}', real=True)))

    @property
    def shape(self):
        return self.M.shape

    @property
    def T(self):
        return SX(self.M.T)

    def __getitem__(self, key):
        if isinstance(key, int) and self.M.shape[1] == 1:
            return _wrap(self.M[key, 0])
        r = self.M[key]
        return _wrap(r)

    def __setitem__(self, key, val):
        v = _mat(val)
        if v.shape == (1, 1) and not isinstance(key, tuple):
            self.M[key] = v[0, 0]
        else:
            self.M[key] = v

    def _bin(self, o, f):
        a, b = self.M, _mat(o)
        if b.shape == (1, 1) and a.shape != (1, 1):
            return SX(a.applyfunc(lambda x: f(x, b[0, 0])))
        if a.shape == (1, 1) and b.shape != (1, 1):
            return SX(b.applyfunc(lambda x: f(a[0, 0], x)))
        return SX(sympy.Matrix(a.shape[0], a.shape[1], lambda i, j: f(a[i, j], b[i, j])))

    def __add__(self, o):
        return self._bin(o, lambda x, y: x + y)

    def __radd__(self, o):
        return _wrap(_mat(o)) + self if not (np.isscalar(o) and o == 0) else self

    def __sub__(self, o):
        return self._bin(o, lambda x, y: x - y)

    def __rsub__(self, o):
        return _wrap(_mat(o))._bin(self, lambda x, y: x - y)

    def __neg__(self):
        return SX(-self.M)

    def __mul__(self, o):
        return self._bin(o, lambda x, y: x * y)

    def __rmul__(self, o):
        return self._bin(o, lambda x, y: y * x)

    def __truediv__(self, o):
        return self._bin(o, lambda x, y: x / y)

    def __matmul__(self, o):
        return SX(self.M * _mat(o))

    def __rmatmul__(self, o):
        return SX(_mat(o) * self.M)


def _cat(args, axis):
    parts = []
    for a in args:
        if isinstance(a, list) and len(a) == 0:
            continue
        parts.append(a)
    if all(not isinstance(a, SX) for a in parts):   # numeric in, numeric out (casadi DM)
        arrs = [np.asarray(a, dtype=np.float64) for a in parts]
        arrs = [a.reshape(-1, 1) if a.ndim == 1 else a for a in arrs]
        return np.concatenate(arrs, axis=axis)
    mats = [_mat(a) for a in parts]
    return SX(sympy.Matrix.hstack(*mats) if axis == 1 else sympy.Matrix.vstack(*mats))


def horzcat(*args):
    return _cat(args, 1)


def vertcat(*args):
    return _cat(args, 0)


def reshape(x, n, m):
    """column-major, as casadi"""
    M = _mat(x)
    flat = [M[i, j] for j in range(M.shape[1]) for i in range(M.shape[0])]
    return SX(sympy.Matrix(m, n, flat).T)


class _Solver:
    def __init__(self, qp):
        self.z = list(_mat(qp['x']))
        self.f = _mat(qp['f'])[0, 0]
        self.g = list(_mat(qp['g']))
        P = _mat(qp['p'])
        self.p = [P[i, j] for i in range(P.shape[0]) for j in range(P.shape[1])]
        self.pshape = P.shape

    def __call__(self, x0=None, lbx=None, ubx=None, lbg=None, ubg=None, p=None):
        pv = np.asarray(p, dtype=np.float64).reshape(self.pshape)
        sub = {s: sympy.Float(float(v)) for s, v in zip(self.p, pv.ravel()) if isinstance(s, sympy.Symbol)}
        n = len(self.z)
        g = [sympy.expand(e.xreplace(sub)) for e in self.g]
        A = np.zeros((len(g), n))
        g0 = np.zeros(len(g))
        zi = {s: i for i, s in enumerate(self.z)}
        for r, e in enumerate(g):
            for term in sympy.Add.make_args(e):
                c, syms = term.as_coeff_mul()
                syms = [s for s in syms if s in zi]
                if not syms:
                    g0[r] += float(term)
                else:
                    assert len(syms) == 1, term
                    A[r, zi[syms[0]]] += float(term / syms[0])
        f = sympy.expand(self.f.xreplace(sub))
        P = np.zeros((n, n))
        q = np.zeros(n)
        r0 = 0.0
        for term in sympy.Add.make_args(f):
            pw = term.as_powers_dict()
            vs = [(s, k) for s, k in pw.items() if s in zi]
            coef = term
            for s, k in vs:
                coef = coef / s ** k
            coef = float(coef)
            if not vs:
                r0 += coef
            elif len(vs) == 1 and vs[0][1] == 1:
                q[zi[vs[0][0]]] += coef
            elif len(vs) == 1 and vs[0][1] == 2:
                P[zi[vs[0][0]], zi[vs[0][0]]] += 2 * coef
            else:
                (s1, _), (s2, _) = vs
                P[zi[s1], zi[s2]] += coef
                P[zi[s2], zi[s1]] += coef
        rec = dict(P=P, q=q, r=r0, A=A, g0=g0, lbg=np.asarray(lbg, float), ubg=np.asarray(ubg, float),
                   lbx=np.asarray(lbx, float), ubx=np.asarray(ubx, float), p=pv)
        RECORD.append(rec)
        z = SOLVER(rec) if SOLVER is not None else np.zeros(n)
        rec['z'] = np.asarray(z, dtype=np.float64)
        return {'x': rec['z'].reshape(-1, 1)}


def qpsol(name, solver, qp, opts=None):
    return _Solver(qp)
