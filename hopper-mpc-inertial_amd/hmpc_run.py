"""Command-line mirror of the reference's run.py (src/run.py:1-27) on the
device Runner (hmpc_runner.Runner):

    python hopper-mpc-inertial_amd/hmpc_run.py 3f [--curve] [--N_run 2000]
                                               [--N 60] [--batch 1] [--out run.npz]

Same positional argument and flags as the reference; the horizon (fixed at 60
in the reference, src/robotrunner.py:46) and the number of robots simulated
at once are extra options.  Plots are out of scope: it prints a summary and
can save the trajectories.
"""
from __future__ import annotations

import argparse
import time

import numpy as np

import hmpc_runner


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument('dyn', help='choose 2f or 3f', choices=['2f', '3f'], type=str)
    ap.add_argument('--curve', help='make the ref traj curved', action='store_true')
    ap.add_argument('--N_run', help='sim run time in ms (integer)', type=int, default=5000)
    ap.add_argument('--N', help='MPC horizon (the reference fixes 60)', type=int, default=60)
    ap.add_argument('--batch', help='robots simulated at once', type=int, default=1)
    ap.add_argument('--out', help='save X_traj / f_hist / s_hist to this .npz', default=None)
    args = ap.parse_args(argv)
    runner = hmpc_runner.Runner(dt=1e-3, dyn=args.dyn, curve=args.curve, N_run=args.N_run, N=args.N,
                                batch=args.batch)
    t0 = time.perf_counter()
    out = runner.run()
    el = time.perf_counter() - t0
    runner.close()
    n_calls = len(out['call_k'])
    print(f'{args.dyn} N={args.N} N_run={args.N_run} curve={args.curve} batch={args.batch}: '
          f'{n_calls} mpcontrol calls ({n_calls + 1} QP solves per robot) in {el:.2f} s; '
          f'final position of robot 0 {np.array2string(out["X_final"][0, :3], precision=4)}')
    if args.out:
        np.savez_compressed(args.out, X_traj=out['X_traj'], f_hist=out['f_hist'], s_hist=out['s_hist'])
    return out


if __name__ == '__main__':
    main()
