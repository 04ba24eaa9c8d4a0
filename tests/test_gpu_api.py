"""Host-side argument checks of the device entry points (hmpc.py): every
tensor handed to the C ABI as a raw pointer is validated first (shape, dtype,
device, contiguity), so a wrong tensor raises instead of becoming an
out-of-bounds GPU access; and the library reports which kernel serves a
context (hmpc_kernel_name)."""
import numpy as np
import pytest
from conftest import DENSE10_3F

torch = pytest.importorskip('torch')

pytestmark = pytest.mark.gpu


@pytest.fixture(scope='module')
def hm():
    if not torch.cuda.is_available():
        pytest.fail('GPU tests need an MI355X (torch.cuda.is_available() is False)')
    import hmpc
    return hmpc


def make(hm, N=10, precision='f64'):
    import hmpc_plan
    c = hmpc_plan.runner_constants()
    return hm.Context('3f', N, t=c['t'], m=c['m'], g=c['g'], mu=1.0, Jinv=c['Jinv'], rh=c['rh'],
                      precision=precision)


def inputs(N, B=4):
    import hmpc_plan
    inst = hmpc_plan.sample_instances(B, N, curve=True, seed=5)
    return {k: torch.from_numpy(np.ascontiguousarray(inst[k])).cuda()
            for k in ('x_in', 'x_lin', 'x_ref', 'pf', 'C', 'mu')}


def test_bad_tensors_raise(hm):
    N = 10
    cx = make(hm, N)
    d = inputs(N)
    args = [d[k] for k in ('x_in', 'x_lin', 'x_ref', 'pf', 'C')]
    cx.solve_device(*args, mu=d['mu'])   # the good call
    bad = [
        (1, d['x_lin'].float()),                  # dtype
        (2, d['x_ref'][:, :N - 1].contiguous()),   # shape
        (3, d['pf'].cpu()),                       # device
        (0, d['x_in'].t().contiguous().t()),      # (shape differs too)
    ]
    for i, t in bad:
        a = list(args)
        a[i] = t
        with pytest.raises(ValueError):
            cx.solve_device(*a, mu=d['mu'])
    with pytest.raises(ValueError):
        cx.solve_device(*args, mu=d['mu'][:2])
    out = dict(u=torch.empty((4, N, 6), dtype=torch.float64, device='cuda'),
               status=torch.empty(4, dtype=torch.int64, device='cuda'))   # wrong status dtype
    with pytest.raises(ValueError):
        cx.solve_device(*args, mu=d['mu'], out=out)
    x_prev = torch.empty((4, N, 12), dtype=torch.float64, device='cuda')   # one row short
    with pytest.raises(ValueError):
        cx.mpcontrol_device(False, d['x_in'], d['x_ref'], d['pf'], d['C'], x_prev)
    cx.close()


def test_kernel_names(hm):
    assert make(hm, 10).kernel_name == DENSE10_3F
    assert make(hm, 20).kernel_name == 'hmpc::ric_kernel<3, 2, 20, 38, 0>'   # 2 waves / SIMD
    assert make(hm, 60).kernel_name == 'hmpc::ric_factor_kernel<3, 60, 47> + hmpc::ric_kernel<3, 1, 60, 47, 2>'   # compile-time N = 60
    assert make(hm, 10, 'f64_riccati').kernel_name == 'hmpc::ric_kernel<3, 2, 0, 0, 0>'
    assert make(hm, 20, 'f64_dense').kernel_name == 'hmpc::solve_kernel<3, 20, double, 0, 0>'
    assert make(hm, 10, 'f64_generic').kernel_name == 'hmpc::wide_kernel<3, double>'
    # fp32 split: the fp64 all-swing class + compacted + full (round 6)
    assert make(hm, 10, 'f32').kernel_name == ('hmpc::swing_kernel<10, 13> + hmpc::solve_kernel<3, 10, float, 48, 13> + '
                                               'hmpc::solve_kernel<3, 10, float, 0, 0>')
    assert make(hm, 10, 'f32_refined').kernel_name == ('hmpc::swing_kernel<10, 13> + '
                                                       'hmpc::solve_kernel<3, 10, float, 48, 13> + '
                                                       'hmpc::solve_kernel<3, 10, float, 0, 0>')
    assert make(hm, 20, 'f32').kernel_name == 'hmpc::wide_kernel<3, float>'   # no fp32 dense build
    assert make(hm, 10, 'f32_generic').kernel_name == 'hmpc::wide_kernel<3, float>'


def test_active_capacity(hm):
    # dense N = 10: the split's compacted kernel holds 13 (LDS for 3 waves /
    # SIMD), the full one 20; Riccati: the largest R that keeps 8 (N <= 24)
    # or 4 workgroups per CU in LDS (hmpc_ric.hip ric_config)
    assert make(hm, 10).active_capacity == 13
    assert make(hm, 20).active_capacity == 38
    assert make(hm, 60).active_capacity == 47
    assert make(hm, 10, 'f64_riccati').active_capacity == 50
    assert make(hm, 10, 'f64_generic').active_capacity == 0


@pytest.mark.parametrize('N', [10, 20])
def test_one_context_two_streams_is_ordered(hm, N):
    """The context's workspaces and self-resetting counters are shared by its
    calls; a solve issued on another stream waits for the context's last one
    (hmpc_capi.cpp order_stream).  Alternating two batches over two streams of
    one context -- overflowing instances included, so the counters are live --
    gives exactly what fresh contexts give."""
    import hmpc_plan as hp
    from test_gpu_overflow import adversarial
    B = 2048
    a = hp.sample_instances(B, N, curve=True, seed=11, mu_sweep=(0.3, 1.2))
    b = adversarial(B, N, 4, 30.0, 5.0)
    dv = lambda inst: {k: torch.from_numpy(np.ascontiguousarray(inst[k])).cuda()
                       for k in ('x_in', 'x_lin', 'x_ref', 'pf', 'C', 'mu')}
    da, db = dv(a), dv(b)
    ref = []
    for d in (da, db):
        cx = make(hm, N)
        o = cx.solve_device(d['x_in'], d['x_lin'], d['x_ref'], d['pf'], d['C'], mu=d['mu'])
        torch.cuda.synchronize()
        ref.append({k: v.cpu().numpy() for k, v in o.items()})
        cx.close()
    cx = make(hm, N)
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    outs = []
    for rep in range(4):
        for d, s in ((da, s1), (db, s2)):
            outs.append(cx.solve_device(d['x_in'], d['x_lin'], d['x_ref'], d['pf'], d['C'], mu=d['mu'],
                                        stream=s.cuda_stream))
    torch.cuda.synchronize()
    cx.close()
    assert (ref[0]['status'] == 0).mean() > 0.9 and (ref[1]['status'] == 0).mean() > 0.5
    for i, o in enumerate(outs):
        r = ref[i % 2]
        for k in ('u', 'x', 'obj', 'status'):
            assert np.array_equal(o[k].cpu().numpy(), r[k]), (i, k)
