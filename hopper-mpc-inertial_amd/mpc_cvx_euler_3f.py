"""Drop-in for the reference module src/mpc_cvx_euler_3f.py (3 world-frame
forces + 3 torques).  ``import mpc_cvx_euler_3f; mpc_cvx_euler_3f.Mpc(...)``
as src/robotrunner.py:5,73,76 does; the QP is solved on the MI355X."""
from hmpc_mpc import MpcBase


class Mpc(MpcBase):
    variant = '3f'
