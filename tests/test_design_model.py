"""The numpy design model of the kernel algorithm (tools/proto_gi.py) agrees
with the independent oracle: condensed Goldfarb-Idnani vs non-condensed
interior point + polish.  Guards the algorithm the HIP kernel implements."""
import numpy as np
import pytest

import hmpc_plan
import proto_gi
from oracle import hmpc_oracle as ho


@pytest.mark.parametrize('variant,N,curve', [('3f', 10, True), ('2f', 10, False), ('3f', 20, False)])
def test_model_matches_oracle(variant, N, curve):
    p = ho.MpcParams.runner(variant, N)
    d = hmpc_plan.sample_instances(6, N, curve=curve, seed=21)
    for i in range(6):
        args = [d[k][i] for k in ('x_in', 'x_lin', 'x_ref', 'pf', 'C')]
        o = ho.solve_instance(p, *args)
        g = proto_gi.solve(p, *args, d['mu'][i])
        assert o['status'] == 'solved' and g['status'] == 0
        assert np.abs(o['u'] - g['u']).max() < 1e-6
        assert abs(o['obj'] - g['obj']) <= 1e-9 * abs(o['obj'])
