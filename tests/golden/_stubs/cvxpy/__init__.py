"""Recording stand-in for cvxpy -- used ONLY by tests/golden/make_golden.py.

cvxpy is not installed in this image (no network).  The reference's
``Mpc.build_qp`` only needs a small modelling surface (Variable indexing,
affine arithmetic with numpy constants, quad_form, comparisons, Problem.solve),
so this stub records the expression tree the reference builds and, at
``Problem.solve`` time, canonicalises it into OSQP standard form
``1/2 z'Pz + q'z + r,  l <= Az <= u`` -- like cvxpy does.

Constants are captured BY REFERENCE (``np.asarray`` without a copy) and read
only at solve time, which is how cvxpy's ``Constant`` treats a float64
ndarray.  This reproduces the ``u_ref`` aliasing of the reference
(SURVEY.md 8a row A4).  Set ``COPY_CONSTANTS = True`` to snapshot constants at
construction time instead (the intended per-stage semantics).

The solve itself is delegated to ``SOLVER`` (set by make_golden.py to the
oracle's exact solver); every canonicalised problem is appended to RECORD.
"""
import numpy as np

OSQP = 'OSQP'
COPY_CONSTANTS = False
SOLVER = None
RECORD = []
_VARS = []


def _const(v):
    a = np.asarray(v)
    if COPY_CONSTANTS:
        a = np.array(a, dtype=np.float64, copy=True)
    return Const(a)


def _as_expr(v):
    return v if isinstance(v, Expr) else _const(v)


class Expr:
    __array_priority__ = 1000
    __array_ufunc__ = None

    def __add__(self, o):
        return Add(self, _as_expr(o))

    def __radd__(self, o):
        return Add(_as_expr(o), self)

    def __sub__(self, o):
        return Add(self, Neg(_as_expr(o)))

    def __rsub__(self, o):
        return Add(_as_expr(o), Neg(self))

    def __neg__(self):
        return Neg(self)

    def __mul__(self, o):
        return Scale(self, o)

    def __rmul__(self, o):
        return Scale(self, o)

    def __rmatmul__(self, M):
        return MatMul(M, self)

    def __le__(self, o):
        return Constraint(self - o, '<=')

    def __ge__(self, o):
        return Constraint(self - o, '>=')

    def __eq__(self, o):
        return Constraint(self - o, '==')

    __hash__ = object.__hash__


class Const(Expr):
    def __init__(self, value):
        self.value_ref = value

    def dim(self):
        return int(np.size(self.value_ref))

    def evaluate(self, nz):
        c = np.asarray(self.value_ref, dtype=np.float64).reshape(-1)
        return np.zeros((c.size, nz)), c.copy()


class VarRef(Expr):
    def __init__(self, var, idx):
        self.var = var
        self.idx = np.atleast_1d(idx)

    def dim(self):
        return self.idx.size

    def evaluate(self, nz):
        A = np.zeros((self.idx.size, nz))
        A[np.arange(self.idx.size), self.var.offset + self.idx] = 1.0
        return A, np.zeros(self.idx.size)


class Add(Expr):
    def __init__(self, a, b):
        self.a, self.b = a, b

    def evaluate(self, nz):
        A1, c1 = self.a.evaluate(nz)
        A2, c2 = self.b.evaluate(nz)
        n = max(c1.size, c2.size)
        A1 = np.broadcast_to(A1, (n, nz)) if c1.size == 1 else A1
        A2 = np.broadcast_to(A2, (n, nz)) if c2.size == 1 else A2
        return A1 + A2, np.broadcast_to(c1, (n,)) + np.broadcast_to(c2, (n,))


class Neg(Expr):
    def __init__(self, a):
        self.a = a

    def evaluate(self, nz):
        A, c = self.a.evaluate(nz)
        return -A, -c


class Scale(Expr):
    def __init__(self, a, s):
        self.a, self.s = a, s

    def evaluate(self, nz):
        A, c = self.a.evaluate(nz)
        return self.s * A, self.s * c


class MatMul(Expr):
    def __init__(self, M, a):
        self.M = np.asarray(M)
        if COPY_CONSTANTS:
            self.M = np.array(self.M, dtype=np.float64, copy=True)
        self.a = a

    def evaluate(self, nz):
        A, c = self.a.evaluate(nz)
        M = np.asarray(self.M, dtype=np.float64)
        return M @ A, M @ c


class Variable:
    def __init__(self, shape):
        self.shape = tuple(shape)
        self.size = int(np.prod(self.shape))
        self.value = None
        self.offset = None
        _VARS.append(self)

    def __getitem__(self, key):
        flat = np.arange(self.size).reshape(self.shape)[key]
        return VarRef(self, flat.reshape(-1) if np.ndim(flat) else flat)


class QuadForm:
    def __init__(self, e, M):
        self.e = e
        self.M = np.asarray(M)

    def terms(self):
        return [self]

    def __add__(self, o):
        return ObjSum(self.terms() + _terms(o))

    __radd__ = __add__


def _terms(o):
    if isinstance(o, (QuadForm, ObjSum)):
        return o.terms()
    if np.isscalar(o) and o == 0:
        return []
    raise TypeError(o)


class ObjSum(QuadForm):
    def __init__(self, ts):
        self.ts = ts

    def terms(self):
        return list(self.ts)


def quad_form(e, M):
    return QuadForm(e, M)


class Constraint:
    def __init__(self, e, op):
        self.e, self.op = e, op


class Minimize:
    def __init__(self, obj):
        self.obj = obj


class Problem:
    def __init__(self, objective, constraints):
        self.objective = objective
        self.constraints = constraints
        self.value = None

    def canonicalize(self):
        found = []

        def walk(e):
            if isinstance(e, VarRef):
                if e.var not in found:
                    found.append(e.var)
            for ch in ('a', 'b', 'e'):
                if hasattr(e, ch) and isinstance(getattr(e, ch), Expr):
                    walk(getattr(e, ch))

        for t in self.objective.obj.terms():
            walk(t.e)
        for con in self.constraints:
            walk(con.e)
        # variables in creation order (x before u, as Mpc.__init__ makes them)
        vars_used = sorted(found, key=lambda v: _VARS.index(v))
        nz = 0
        for v in vars_used:
            v.offset = nz
            nz += v.size
        P = np.zeros((nz, nz))
        q = np.zeros(nz)
        r = 0.0
        for t in self.objective.obj.terms():
            A, c = t.e.evaluate(nz)
            M = np.asarray(t.M, dtype=np.float64)
            P += 2 * A.T @ M @ A
            q += 2 * A.T @ M @ c
            r += c @ M @ c
        rows, lo, hi = [], [], []
        for con in self.constraints:
            A, c = con.e.evaluate(nz)
            for i in range(A.shape[0]):
                rows.append(A[i])
                if con.op == '<=':
                    lo.append(-np.inf); hi.append(-c[i])
                elif con.op == '>=':
                    lo.append(-c[i]); hi.append(np.inf)
                else:
                    lo.append(-c[i]); hi.append(-c[i])
        return vars_used, dict(P=P, q=q, r=r, A=np.array(rows), l=np.array(lo), u=np.array(hi))

    def solve(self, solver=None, **kw):
        vars_used, qp = self.canonicalize()
        sol = SOLVER(qp['P'], qp['q'], qp['A'], qp['l'], qp['u'])
        RECORD.append(dict(qp=qp, sol=sol))
        if sol['x'] is None:
            for v in vars_used:
                v.value = None
            return None
        z = sol['x']
        for v in vars_used:
            v.value = z[v.offset:v.offset + v.size].reshape(v.shape).copy()
        self.value = 0.5 * z @ qp['P'] @ z + qp['q'] @ z + qp['r']
        return self.value
