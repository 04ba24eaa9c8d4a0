"""Stand-in for transforms3d (absent here) -- used ONLY by make_golden.py.

The reference only calls ``transforms3d.euler.quat2euler(Q, axes='rzyx')``
(src/utils.py:57); see euler.py for the restated algorithm.
"""
from . import euler  # noqa: F401
