"""Run the reference Runner's default configuration (3f, N = 60,
N_run = 2000; run.py 3f) through the device Runner and report the first
failing MPC call, if any."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'hopper-mpc-inertial_amd'))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

import hmpc_runner  # noqa: E402

curve = '--curve' in sys.argv
r = hmpc_runner.Runner(dyn='3f', curve=curve, N_run=2000, N=60, batch=1)
t = time.time()
try:
    out = r.run()
    print('completed', out['X_traj'].shape, 'in %.2fs' % (time.time() - t), 'final', out['X_final'][0, :3])
except Exception as e:  # QP FAILED
    print('failed after %.2fs:' % (time.time() - t), e)
