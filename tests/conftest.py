import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, 'hopper-mpc-inertial_amd')
GOLDEN = os.path.join(ROOT, 'tests', 'golden')
# the default build's N = 10 3f dense dispatch: the split's persistent class
# kernels (compacted nf <= 48, then the full class), as hmpc_kernel_name
# reports them (build.sh CMP)
DENSE10_3F = 'hmpc::swing_kernel<10, 13> + hmpc::solve_kernel<3, 10, double, 48, 13> + hmpc::solve_kernel<3, 10, double, 0, 0>'
# longest-first order (small batches): the all-swing windows stay in the compacted class
DENSE10_3F_LPT = DENSE10_3F.split(' + ', 1)[1]
for p in (PKG, ROOT, os.path.join(ROOT, 'tools')):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line('markers', 'gpu: needs an MI355X (runs through libhmpc.so)')


@pytest.fixture(scope='session')
def golden_dir():
    return GOLDEN
