"""Drop-in for the reference module src/mpc_cvx_euler_2f.py (planar: body-
frame force with fy = 0).  Used as src/robotrunner.py:6,71,76 does; the QP is
solved on the MI355X."""
from hmpc_mpc import MpcBase


class Mpc(MpcBase):
    variant = '2f'
