"""Wall time of the device Runner (hmpc_runner.Runner.run: plan + gait +
100 MPC periods of mpcontrol_plan + plant) for the reference's configs[0]
(run.py 3f --N_run=2000, N = 60) at batch 1 and a few batch sizes.
python tools/runner_time.py [graph] [B ...]     (graph: timed run = a replay of the
captured run, hmpc_runner.Runner.run(graph=True); robot counts, default 1 256 4096)"""
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'hopper-mpc-inertial_amd'))
import hmpc_runner  # noqa: E402

graph = 'graph' in sys.argv[1:]
res = {}
batches = [int(x) for x in sys.argv[1:] if x.isdigit()] or [1, 256, 4096]
for B in batches:
    r = hmpc_runner.Runner(dt=1e-3, dyn='3f', curve=False, N_run=2000, N=60, batch=B)
    kw = dict(record=False)
    if graph:
        kw['graph'] = True
    # warm (workspaces, code objects); graph: the full-length run captures
    r.run(n_periods=None if graph else 2, **kw)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    out = r.run(**kw)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    r.close()
    res[B] = {'seconds': el, 'robot_steps_per_s': B * 2000 / el, 'mpc_solves_per_s': B * 101 / el,
              'all_solved': bool((out['status'] == 0).all())}
print(json.dumps({'graph': graph, 'runner_N60_2000_steps': res}, indent=1))
