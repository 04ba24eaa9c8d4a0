"""Product-side planner (hmpc_plan.py) against the reference's own planner output.

plan.npz holds ``Runner.path_plan_init`` / ``gait_map`` results recorded from
src/robotrunner.py:166-230 (straight and --curve, N_run = 2000, N = 60).
"""
import os

import numpy as np

import hmpc_plan


def test_path_plan_matches_reference(golden_dir):
    d = np.load(os.path.join(golden_dir, 'plan.npz'))
    for curve in (False, True):
        tag = 'curve' if curve else 'straight'
        _, x_ref, pf_ref = hmpc_plan.runner_plan(curve=curve, N_run=2000)
        assert x_ref.shape == (3200, 12)
        assert np.array_equal(x_ref, d[f'{tag}_x_ref'])
        assert np.array_equal(pf_ref, d[f'{tag}_pf_ref'])


def test_gait_map_matches_reference(golden_dir):
    d = np.load(os.path.join(golden_dir, 'plan.npz'))
    cfg = hmpc_plan.RunnerConfig()
    C = np.array([hmpc_plan.gait_map(cfg, 10, 0.02, t, 0) for t in d['gait_ts']])
    assert np.array_equal(C, d['gait_C10'])


def test_sampler_is_deterministic_and_shaped():
    a = hmpc_plan.sample_instances(257, 10, curve=True, seed=3)
    b = hmpc_plan.sample_instances(257, 10, curve=True, seed=3)
    for k in a:
        assert np.array_equal(a[k], b[k])
    assert a['x_lin'].shape == (257, 11, 12) and a['C'].shape == (257, 10)
    assert np.array_equal(a['x_lin'][:, 0], a['x_in'])
    assert np.array_equal(a['x_lin'][:, 1:], a['x_ref'])
    m = hmpc_plan.sample_instances(64, 20, mu_sweep=(0.3, 1.2), seed=1)['mu']
    assert m.min() >= 0.3 and m.max() <= 1.2


def test_sampler_shards_reproduce_the_global_batch():
    """Instance i depends only on (seed, i): shards drawn by separate ranks
    concatenate to the single-process batch."""
    B = 3 * hmpc_plan.BLOCK + 100
    full = hmpc_plan.sample_instances(B, 10, curve=True, seed=11, mu_sweep=(0.3, 1.2))
    cuts = [0, 1000, hmpc_plan.BLOCK, 2 * hmpc_plan.BLOCK + 7, B]
    for lo, hi in zip(cuts[:-1], cuts[1:]):
        part = hmpc_plan.sample_instances(hi - lo, 10, curve=True, seed=11, mu_sweep=(0.3, 1.2),
                                          start=lo)
        for k in full:
            assert np.array_equal(part[k], full[k][lo:hi]), (k, lo, hi)
    assert hmpc_plan.sample_instances(0, 10)['x_in'].shape == (0, 12)
