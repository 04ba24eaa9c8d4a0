"""TEST INFRASTRUCTURE ONLY -- the CPU oracle for the batched MPC/QP solve path.

Nothing in the product path (``hopper-mpc-inertial_amd/``) may import, link or
execute anything under ``oracle/``.  Only ``tests/``, ``__graft_entry__.smoke()``
and the ``cpu_baseline`` leg of ``bench.py`` use it, and only as the checker.

Contents
--------
``hmpc_oracle``  numpy restatement of the reference's problem construction
                 (``Mpc.gen_dt_dynamics`` / ``Mpc.build_qp`` / ``Mpc.mpcontrol``
                 of ``src/mpc_cvx_euler_{2f,3f}.py``) into OSQP standard form.
``qp_exact``     an exact fp64 QP solve of that standard form (interior point
                 to 1e-12, then an active-set polish and a KKT certificate).
                 It stands in for cvxpy+OSQP, which are absent from this image.
``hmpc_port.c`` a plain-C restatement of the same construction, condensed
  / ``port``     densely and solved exactly by a classic Goldfarb-Idnani dual
                 active set (``make -C oracle`` -> libhmpc_port.so, ctypes
                 binding in ``port.py``): the second checker and the
                 ``cpu_baseline`` "port" timed by bench.py (OpenMP).

The synthetic-instance planner (``Runner.path_plan_init`` / ``gait_map``
restated) lives on the product side, ``hopper-mpc-inertial_amd/hmpc_plan.py``,
pinned by tests/test_plan.py against the reference's recorded plan.

Pinning: the problem data is pinned bit-for-bit (to a few ulps) against
fixtures recorded from the reference's OWN ``gen_dt_dynamics``/``build_qp``
(``tests/golden/make_golden.py`` imports /root/reference with a recording
cvxpy stub).  The solutions are pinned by KKT certificates; cvxpy/OSQP could
not be run here (not installed, no network), so "u* of cvxpy/OSQP" is taken
to mean the exact optimum of the reference-built QP.
"""
