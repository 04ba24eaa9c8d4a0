"""Restatement of transforms3d.euler.quat2euler for the axes the reference uses.

transforms3d (Gohlke/Brett, BSD) converts a quaternion to a matrix
(``quaternions.quat2mat``: s = 2/|q|^2, identity below eps) and the matrix to
Euler angles (``euler.mat2euler`` with the 'rzyx' axis tuple (0, 0, 0, 1):
first axis x, even parity, no repetition, rotating frame => the static 'sxyz'
angles with ax/az swapped).  Only 'rzyx' is implemented -- it is the only
axis string in the reference (src/utils.py:57).
"""
import math

import numpy as np

_FLOAT_EPS = np.finfo(np.float64).eps
_EPS4 = _FLOAT_EPS * 4.0


def quat2mat(q):
    w, x, y, z = q
    Nq = w * w + x * x + y * y + z * z
    if Nq < _FLOAT_EPS:
        return np.eye(3)
    s = 2.0 / Nq
    X = x * s
    Y = y * s
    Z = z * s
    wX = w * X; wY = w * Y; wZ = w * Z
    xX = x * X; xY = x * Y; xZ = x * Z
    yY = y * Y; yZ = y * Z; zZ = z * Z
    return np.array(
        [[1.0 - (yY + zZ), xY - wZ, xZ + wY],
         [xY + wZ, 1.0 - (xX + zZ), yZ - wX],
         [xZ - wY, yZ + wX, 1.0 - (xX + yY)]])


def mat2euler(mat, axes='rzyx'):
    if axes != 'rzyx':
        raise NotImplementedError(axes)
    i, j, k = 0, 1, 2
    M = np.asarray(mat, dtype=np.float64)[:3, :3]
    cy = math.sqrt(M[i, i] * M[i, i] + M[j, i] * M[j, i])
    if cy > _EPS4:
        ax = math.atan2(M[k, j], M[k, k])
        ay = math.atan2(-M[k, i], cy)
        az = math.atan2(M[j, i], M[i, i])
    else:
        ax = math.atan2(-M[j, k], M[j, j])
        ay = math.atan2(-M[k, i], cy)
        az = 0.0
    # rotating frame: swap first and last
    ax, az = az, ax
    return ax, ay, az


def quat2euler(quaternion, axes='rzyx'):
    return mat2euler(quat2mat(quaternion), axes)
