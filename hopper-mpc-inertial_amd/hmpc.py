"""ctypes binding of libhmpc.so -- the C ABI in include/hmpc.h.

This is the host side of the drop-in boundary: plain pointers and sizes go
through the C ABI, PyTorch is used only as a device-memory/stream provider
(``torch.Tensor.data_ptr()``) when the caller keeps its batch on the GPU.
There is no CPU fallback anywhere in this module: if the shared library or a
GPU is missing, every entry point raises.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get('HMPC_LIB', os.path.join(HERE, 'libhmpc.so'))

HMPC_OK = 0
ERRORS = {-1: 'HMPC_ERR_ARG', -2: 'HMPC_ERR_UNSUPPORTED', -3: 'HMPC_ERR_HIP', -4: 'HMPC_ERR_NOMEM'}
STATUS = {0: 'solved', 1: 'max_iter', 2: 'primal_infeasible', 3: 'numerical'}
VARIANTS = {'3f': 3, '2f': 2, 'cas': 4, 3: 3, 2: 2, 4: 4}
UREF = {'aliased': 0, 'per_stage': 1}
PRECISION = {'f64': 0, 'f32': 1, 'f64_generic': 2, 'f64_riccati': 3, 'f64_dense': 4, 'f32_generic': 5,
             'f32_refined': 6}
ORDER = {'auto': 0, 'index': 1, 'longest_first': 2}

# symbol -> (restype, argtypes); every symbol declared in include/hmpc.h
_D = ctypes.POINTER(ctypes.c_double)
_I32 = ctypes.POINTER(ctypes.c_int32)
_VP = ctypes.c_void_p
SIGNATURES = {
    'hmpc_version': (ctypes.c_int, []),
    'hmpc_supported_horizons': (ctypes.c_int, [ctypes.c_int, ctypes.POINTER(ctypes.c_int), ctypes.c_int]),
    'hmpc_create': (ctypes.c_int, [ctypes.POINTER(_VP), ctypes.c_int, ctypes.c_int, ctypes.c_double,
                                   ctypes.c_double, ctypes.c_double, ctypes.c_double, _D, _D,
                                   ctypes.c_int, ctypes.c_int]),
    'hmpc_destroy': (ctypes.c_int, [_VP]),
    'hmpc_solve_batch': (ctypes.c_int, [_VP, ctypes.c_int64] + [_VP] * 11 + [_VP]),
    'hmpc_solve_batch_stats': (ctypes.c_int, [_VP, ctypes.c_int64] + [_VP] * 12 + [_VP]),
    'hmpc_set_refinement': (ctypes.c_int, [_VP, ctypes.c_int]),
    'hmpc_set_order': (ctypes.c_int, [_VP, ctypes.c_int]),
    'hmpc_solve_batch_host': (ctypes.c_int, [_VP, ctypes.c_int64] + [_VP] * 11),
    'hmpc_mpcontrol_batch': (ctypes.c_int, [_VP, ctypes.c_int64, ctypes.c_int] + [_VP] * 10 + [_VP]),
    'hmpc_mpcontrol_plan_batch': (ctypes.c_int, [_VP, ctypes.c_int64, ctypes.c_int, _VP, _VP, _VP,
                                                 ctypes.c_int64, ctypes.c_int64, ctypes.c_int64,
                                                 ctypes.c_int, _VP, ctypes.c_int64]
                                  + [_VP] * 6 + [_VP]),
    'hmpc_plant_batch': (ctypes.c_int, [_VP, ctypes.c_int64, ctypes.c_int, ctypes.c_double, _D, _VP,
                                        _VP, ctypes.c_int64, _VP, ctypes.c_int64, ctypes.c_int64,
                                        _VP, _VP, _VP]),
    'hmpc_convert_batch': (ctypes.c_int, [_VP, ctypes.c_int64, _VP, _VP, _VP]),
    'hmpc_plan_batch': (ctypes.c_int, [_VP, ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.c_double,
                                       ctypes.c_int, ctypes.c_double, ctypes.c_double, ctypes.c_double,
                                       ctypes.c_int, _VP, _VP, _VP, _VP, _VP, _VP]),
    'hmpc_gait_batch': (ctypes.c_int, [_VP, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_double,
                                       ctypes.c_double, ctypes.c_double, ctypes.c_double, ctypes.c_double,
                                       ctypes.c_double, _VP, _VP, _VP]),
    'hmpc_set_precision': (ctypes.c_int, [_VP, ctypes.c_int]),
    'hmpc_last_error': (ctypes.c_char_p, [_VP]),
    'hmpc_kernel_name': (ctypes.c_char_p, [_VP]),
    'hmpc_active_capacity': (ctypes.c_int, [_VP]),
    'hmpc_overflow_total': (ctypes.c_int, [_VP, _VP]),
    'hmpc_time_solve_batch': (ctypes.c_int, [_VP, ctypes.c_int64] + [_VP] * 11
                              + [ctypes.c_int, _VP, ctypes.POINTER(ctypes.c_double)]),
}

_lib = None


def load(path: str | None = None):
    """Load libhmpc.so (built in-tree by build.sh); raises if absent."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    p = path or LIB_PATH
    if not os.path.exists(p):
        raise RuntimeError(f'libhmpc.so not found at {p}: run hopper-mpc-inertial_amd/build.sh '
                           '(there is no CPU fallback)')
    lib = ctypes.CDLL(p)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if path is None:
        _lib = lib
    return lib


def supported_horizons(variant='3f'):
    lib = load()
    buf = (ctypes.c_int * 16)()
    n = lib.hmpc_supported_horizons(VARIANTS[variant], buf, 16)
    return [buf[i] for i in range(min(n, 16))]


def _ptr(a):
    if a is None:
        return None
    if hasattr(a, 'data_ptr'):
        return ctypes.c_void_p(a.data_ptr())
    return a.ctypes.data_as(ctypes.c_void_p)


class HmpcError(RuntimeError):
    pass


def _check_tensor(t, shape, name, device, dtype='float64', optional=False):
    """A device argument must be a contiguous CUDA tensor of exactly this
    shape and dtype on the context's device: the C ABI takes raw pointers, so
    anything else would be an out-of-bounds access or a silent misread."""
    import torch
    if t is None:
        if optional:
            return
        raise ValueError(f'{name} is required')
    dt = torch.float64 if dtype == 'float64' else torch.int32
    if not isinstance(t, torch.Tensor) or not t.is_cuda:
        raise ValueError(f'{name} must be a CUDA tensor')
    if t.device.index != device:
        raise ValueError(f'{name} is on cuda:{t.device.index}, the context on cuda:{device}')
    if t.dtype != dt:
        raise ValueError(f'{name} must be {dtype}, got {t.dtype}')
    if tuple(t.shape) != tuple(shape):
        raise ValueError(f'{name} must have shape {tuple(shape)}, got {tuple(t.shape)}')
    if not t.is_contiguous():
        raise ValueError(f'{name} must be contiguous')


def _check_out(out, B, N, device, need_x=False):
    _check_tensor(out.get('u'), (B, N, 6), "out['u']", device)
    _check_tensor(out.get('x'), (B, N + 1, 12), "out['x']", device, optional=not need_x)
    _check_tensor(out.get('obj'), (B,), "out['obj']", device, optional=True)
    _check_tensor(out.get('status'), (B,), "out['status']", device, dtype='int32')
    _check_tensor(out.get('iters'), (B,), "out['iters']", device, dtype='int32', optional=True)
    _check_tensor(out.get('active'), (B,), "out['active']", device, dtype='int32', optional=True)


class Context:
    """One device-side ``Mpc`` (src/mpc_cvx_euler_3f.py:12-39) for a fixed
    (variant, N) and the Runner's physical constants."""

    def __init__(self, variant='3f', N=10, t=0.02, m=7.5, g=9.807, mu=1.0, Jinv=None, rh=None,
                 uref_mode='aliased', device=0, precision='f64'):
        lib = load()
        if Jinv is None or rh is None:
            raise ValueError('Jinv and rh are required')
        self.variant = VARIANTS[variant]
        self.N = int(N)
        self.device = int(device)
        J = np.ascontiguousarray(np.asarray(Jinv, dtype=np.float64).reshape(9))
        r = np.ascontiguousarray(np.asarray(rh, dtype=np.float64).reshape(3))
        h = ctypes.c_void_p()
        rc = lib.hmpc_create(ctypes.byref(h), self.variant, self.N, float(t), float(m), float(g),
                             float(mu), J.ctypes.data_as(_D), r.ctypes.data_as(_D),
                             UREF[uref_mode], self.device)
        if rc != HMPC_OK:
            raise HmpcError(f'hmpc_create({variant}, N={N}) failed: {ERRORS.get(rc, rc)}')
        self._h = h
        self._lib = lib
        if precision != 'f64':
            self._check(lib.hmpc_set_precision(h, PRECISION[precision]), 'hmpc_set_precision')

    def set_refinement(self, corrections):
        """fp64 corrections of precision 'f32_refined' (hmpc_set_refinement)."""
        self._check(self._lib.hmpc_set_refinement(self._h, int(corrections)), 'hmpc_set_refinement')

    def set_order(self, order):
        """Instance order of later solves (hmpc_set_order): 'auto' (longest-first
        for small batches), 'index' or 'longest_first'.  Results do not depend on it."""
        self._check(self._lib.hmpc_set_order(self._h, ORDER[order]), 'hmpc_set_order')

    @property
    def kernel_name(self):
        """The solve kernel this context runs on (hmpc_kernel_name)."""
        return self._lib.hmpc_kernel_name(self._h).decode()

    @property
    def active_capacity(self):
        """Active-set capacity of the main pass (hmpc_active_capacity)."""
        return int(self._lib.hmpc_active_capacity(self._h))

    @property
    def overflow_total(self):
        """Instances the overflow pass re-solved on this context so far
        (hmpc_overflow_total; waits for the last solve)."""
        v = ctypes.c_int64(0)
        self._check(self._lib.hmpc_overflow_total(self._h, ctypes.byref(v)), 'hmpc_overflow_total')
        return int(v.value)

    def close(self):
        if getattr(self, '_h', None):
            self._lib.hmpc_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc, what):
        if rc != HMPC_OK:
            msg = self._lib.hmpc_last_error(self._h).decode()
            raise HmpcError(f'{what} failed: {ERRORS.get(rc, rc)} {msg}')

    # -- host arrays (numpy): synchronous ------------------------------------
    def solve_host(self, x_in, x_lin, x_ref, pf, C, mu=None):
        N = self.N
        c = lambda a: np.ascontiguousarray(np.asarray(a, dtype=np.float64))  # noqa: E731
        x_in, x_lin, x_ref, pf, C = c(x_in), c(x_lin), c(x_ref), c(pf), c(C)
        B = x_in.shape[0]
        assert x_in.shape == (B, 12) and x_lin.shape == (B, N + 1, 12)
        assert x_ref.shape == (B, N, 12) and pf.shape == (B, N, 3) and C.shape == (B, N)
        mu_a = None if mu is None else c(np.broadcast_to(np.asarray(mu, dtype=np.float64), (B,)))
        u = np.empty((B, N, 6))
        x = np.empty((B, N + 1, 12))
        obj = np.empty(B)
        st = np.empty(B, dtype=np.int32)
        it = np.empty(B, dtype=np.int32)
        rc = self._lib.hmpc_solve_batch_host(self._h, B, _ptr(x_in), _ptr(x_lin), _ptr(x_ref),
                                             _ptr(pf), _ptr(C), _ptr(mu_a), _ptr(u), _ptr(x),
                                             _ptr(obj), _ptr(st), _ptr(it))
        self._check(rc, 'hmpc_solve_batch_host')
        return dict(u=u, x=x, obj=obj, status=st, iters=it)

    # -- device tensors (torch, already on this context's GPU): async --------
    def solve_device(self, x_in, x_lin, x_ref, pf, C, mu=None, out=None, stream=None):
        import torch
        N = self.N
        B = x_in.shape[0]
        for t_, shp, nm in ((x_in, (B, 12), 'x_in'), (x_lin, (B, N + 1, 12), 'x_lin'),
                            (x_ref, (B, N, 12), 'x_ref'), (pf, (B, N, 3), 'pf'), (C, (B, N), 'C')):
            _check_tensor(t_, shp, nm, self.device)
        _check_tensor(mu, (B,), 'mu', self.device, optional=True)
        if out is None:
            dev = x_in.device
            out = dict(u=torch.empty((B, N, 6), dtype=torch.float64, device=dev),
                       x=torch.empty((B, N + 1, 12), dtype=torch.float64, device=dev),
                       obj=torch.empty(B, dtype=torch.float64, device=dev),
                       status=torch.empty(B, dtype=torch.int32, device=dev),
                       iters=torch.empty(B, dtype=torch.int32, device=dev))
        _check_out(out, B, N, self.device)
        s = stream if stream is not None else torch.cuda.current_stream(x_in.device).cuda_stream
        # out['active'] (optional, int32 [B]): each instance's final active-set size
        rc = self._lib.hmpc_solve_batch_stats(self._h, B, _ptr(x_in), _ptr(x_lin), _ptr(x_ref), _ptr(pf),
                                              _ptr(C), _ptr(mu), _ptr(out['u']), _ptr(out.get('x')),
                                              _ptr(out.get('obj')), _ptr(out['status']),
                                              _ptr(out.get('iters')), _ptr(out.get('active')),
                                              ctypes.c_void_p(s))
        self._check(rc, 'hmpc_solve_batch_stats')
        return out

    def mpcontrol_device(self, init, x_in, x_ref, pf, C, x_prev, mu=None, out=None, stream=None):
        """Batched ``Mpc.mpcontrol`` on device tensors; x_prev (B,N+1,12) is
        read (init=False) and overwritten with the new x*."""
        import torch
        N = self.N
        B = x_in.shape[0]
        for t_, shp, nm in ((x_in, (B, 12), 'x_in'), (x_ref, (B, N, 12), 'x_ref'), (pf, (B, N, 3), 'pf'),
                            (C, (B, N), 'C'), (x_prev, (B, N + 1, 12), 'x_prev')):
            _check_tensor(t_, shp, nm, self.device)
        _check_tensor(mu, (B,), 'mu', self.device, optional=True)
        if out is None:
            dev = x_in.device
            out = dict(u=torch.empty((B, N, 6), dtype=torch.float64, device=dev),
                       obj=torch.empty(B, dtype=torch.float64, device=dev),
                       status=torch.empty(B, dtype=torch.int32, device=dev),
                       iters=torch.empty(B, dtype=torch.int32, device=dev))
        _check_out(out, B, N, self.device)
        s = stream if stream is not None else torch.cuda.current_stream(x_in.device).cuda_stream
        rc = self._lib.hmpc_mpcontrol_batch(self._h, B, 1 if init else 0, _ptr(x_in), _ptr(x_ref),
                                            _ptr(pf), _ptr(C), _ptr(mu), _ptr(x_prev),
                                            _ptr(out['u']), _ptr(out.get('obj')),
                                            _ptr(out['status']), _ptr(out.get('iters')),
                                            ctypes.c_void_p(s))
        self._check(rc, 'hmpc_mpcontrol_batch')
        return out

    def mpcontrol_plan_device(self, init, x_in, x_ref_plan, pf_plan, k, mpc_factor, C, x_prev,
                              mu=None, out=None, stream=None):
        """The Runner's ``mpcontrol`` call (src/robotrunner.py:98-107) for B
        robots, reading path_plan_grab(plan, k) in place from a device plan:
        x_ref_plan (T,12) / pf_plan (T,3) shared by the batch, or (B,T,12) /
        (B,T,3) one per robot.  C is (N,) shared or (B,N)."""
        import torch
        N = self.N
        B = x_in.shape[0]
        shared = x_ref_plan.dim() == 2
        T = x_ref_plan.shape[-2]
        for t_, last in ((x_ref_plan, 12), (pf_plan, 3)):
            if t_.dtype != torch.float64 or not t_.is_cuda or not t_.is_contiguous() \
                    or t_.shape[-1] != last or t_.shape[-2] != T or (t_.dim() == 2) != shared:
                raise ValueError('plans must be contiguous float64 cuda tensors (T,12)/(T,3) '
                                 'or (B,T,12)/(B,T,3)')
        if not shared and x_ref_plan.shape[0] != B:
            raise ValueError('per-robot plans need a leading batch dimension B')
        for t_, nm in ((x_ref_plan, 'x_ref_plan'), (pf_plan, 'pf_plan')):
            _check_tensor(t_, tuple(t_.shape), nm, self.device)
        _check_tensor(x_in, (B, 12), 'x_in', self.device)
        _check_tensor(x_prev, (B, N + 1, 12), 'x_prev', self.device)
        _check_tensor(C, (N,) if C.dim() == 1 else (B, N), 'C', self.device)
        _check_tensor(mu, (B,), 'mu', self.device, optional=True)
        C_bs = 0 if C.dim() == 1 else N
        if out is None:
            dev = x_in.device
            out = dict(u=torch.empty((B, N, 6), dtype=torch.float64, device=dev),
                       obj=torch.empty(B, dtype=torch.float64, device=dev),
                       status=torch.empty(B, dtype=torch.int32, device=dev),
                       iters=torch.empty(B, dtype=torch.int32, device=dev))
        _check_out(out, B, N, self.device)
        s = stream if stream is not None else torch.cuda.current_stream(x_in.device).cuda_stream
        rc = self._lib.hmpc_mpcontrol_plan_batch(
            self._h, B, 1 if init else 0, _ptr(x_in), _ptr(x_ref_plan), _ptr(pf_plan), T,
            0 if shared else T, int(k), int(mpc_factor), _ptr(C), C_bs, _ptr(mu), _ptr(x_prev),
            _ptr(out['u']), _ptr(out.get('obj')), _ptr(out['status']), _ptr(out.get('iters')),
            ctypes.c_void_p(s))
        self._check(rc, 'hmpc_mpcontrol_plan_batch')
        return out

    def plant_device(self, X, U, U_bstride, pf, pf_bstride, pf_sstride, n_steps, dt, J,
                     X_hist=None, x_out=None, stream=None):
        """n_steps RK4 plant steps (src/robotrunner.py:126-164) on X (B,13)
        in place; see hmpc_plant_batch for the strides."""
        import torch
        B = X.shape[0]
        _check_tensor(X, (B, 13), 'X', self.device)
        for t_, nm in ((U, 'U'), (pf, 'pf')):
            _check_tensor(t_, tuple(t_.shape), nm, self.device)
        if U.numel() < (B - 1) * int(U_bstride) + 6:
            raise ValueError('U is too small for B rows at U_bstride')
        if pf.numel() < (B - 1) * int(pf_bstride) + (int(n_steps) - 1) * int(pf_sstride) + 3:
            raise ValueError('pf is too small for B robots x n_steps at the given strides')
        _check_tensor(X_hist, (B, int(n_steps), 13), 'X_hist', self.device, optional=True)
        _check_tensor(x_out, (B, 12), 'x_out', self.device, optional=True)
        Jh = np.ascontiguousarray(np.asarray(J, dtype=np.float64).reshape(9))
        s = stream if stream is not None else torch.cuda.current_stream(X.device).cuda_stream
        rc = self._lib.hmpc_plant_batch(self._h, B, int(n_steps), float(dt), Jh.ctypes.data_as(_D),
                                        _ptr(X), _ptr(U), int(U_bstride), _ptr(pf), int(pf_bstride),
                                        int(pf_sstride), _ptr(X_hist), _ptr(x_out),
                                        ctypes.c_void_p(s))
        self._check(rc, 'hmpc_plant_batch')

    def plan_device(self, x_in, xf, N_run, N_k, dt, curve, t_p, phi_switch, t_start, step_adjustment,
                    stream=None):
        """Runner.path_plan_init (src/robotrunner.py:182-226) for B robots on
        the device (hmpc_plan_batch): x_in / xf (B,12) start and goal states.
        Returns x_ref (B,T,12), pf_ref (B,T,3) and the gait map C (T,),
        T = N_run + N_k."""
        import torch
        B = x_in.shape[0]
        _check_tensor(x_in, (B, 12), 'x_in', self.device)
        _check_tensor(xf, (B, 12), 'xf', self.device)
        T = int(N_run) + int(N_k)
        dev = x_in.device
        x_ref = torch.empty((B, T, 12), dtype=torch.float64, device=dev)
        pf_ref = torch.empty((B, T, 3), dtype=torch.float64, device=dev)
        C = torch.empty(T, dtype=torch.float64, device=dev)
        s = stream if stream is not None else torch.cuda.current_stream(dev).cuda_stream
        rc = self._lib.hmpc_plan_batch(self._h, B, int(N_run), int(N_k), float(dt), 1 if curve else 0,
                                       float(t_p), float(phi_switch), float(t_start), int(step_adjustment),
                                       _ptr(x_in), _ptr(xf), _ptr(x_ref), _ptr(pf_ref), _ptr(C),
                                       ctypes.c_void_p(s))
        self._check(rc, 'hmpc_plan_batch')
        return x_ref, pf_ref, C

    def gait_device(self, n_steps, mpc_factor, N, dt, mpc_dt, t_p, phi_switch, t_start, t0=0.0,
                    device=None, stream=None):
        """The Runner loop's gait schedule (hmpc_gait_batch): C_calls
        (n_calls, N) = gait_map(N, mpc_dt, t_k, t0) at every MPC call and s_hist
        (n_steps,) = gait_scheduler(t_k, t0) per low-level step."""
        import torch
        dev = torch.device('cuda', self.device) if device is None else device
        n_calls = (int(n_steps) + int(mpc_factor) - 1) // int(mpc_factor)
        C = torch.empty((n_calls, int(N)), dtype=torch.float64, device=dev)
        s_hist = torch.empty(int(n_steps), dtype=torch.float64, device=dev)
        s = stream if stream is not None else torch.cuda.current_stream(dev).cuda_stream
        rc = self._lib.hmpc_gait_batch(self._h, int(n_steps), int(mpc_factor), int(N), float(dt),
                                       float(mpc_dt), float(t_p), float(phi_switch), float(t_start),
                                       float(t0), _ptr(C), _ptr(s_hist), ctypes.c_void_p(s))
        self._check(rc, 'hmpc_gait_batch')
        return C, s_hist

    def convert_device(self, X, x, stream=None):
        """x (B,12) = convert(X (B,13)) (src/robotrunner.py:19-28)."""
        import torch
        _check_tensor(X, (X.shape[0], 13), 'X', self.device)
        _check_tensor(x, (X.shape[0], 12), 'x', self.device)
        s = stream if stream is not None else torch.cuda.current_stream(X.device).cuda_stream
        rc = self._lib.hmpc_convert_batch(self._h, X.shape[0], _ptr(X), _ptr(x), ctypes.c_void_p(s))
        self._check(rc, 'hmpc_convert_batch')

    def time_solve_device(self, x_in, x_lin, x_ref, pf, C, mu, out, reps, stream):
        """Mean kernel time (ms) over `reps` back-to-back launches, measured
        with HIP events on `stream` inside the library."""
        B, N = x_in.shape[0], self.N
        for t_, shp, nm in ((x_in, (B, 12), 'x_in'), (x_lin, (B, N + 1, 12), 'x_lin'),
                            (x_ref, (B, N, 12), 'x_ref'), (pf, (B, N, 3), 'pf'), (C, (B, N), 'C')):
            _check_tensor(t_, shp, nm, self.device)
        _check_tensor(mu, (B,), 'mu', self.device, optional=True)
        _check_out(out, B, N, self.device)
        ms = ctypes.c_double()
        rc = self._lib.hmpc_time_solve_batch(self._h, x_in.shape[0], _ptr(x_in), _ptr(x_lin),
                                             _ptr(x_ref), _ptr(pf), _ptr(C), _ptr(mu),
                                             _ptr(out['u']), _ptr(out.get('x')),
                                             _ptr(out.get('obj')), _ptr(out['status']),
                                             _ptr(out.get('iters')), int(reps),
                                             ctypes.c_void_p(stream), ctypes.byref(ms))
        self._check(rc, 'hmpc_time_solve_batch')
        return ms.value
