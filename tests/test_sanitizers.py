"""Host-side sanitizers: AddressSanitizer +
UndefinedBehaviorSanitizer over

* the oracle's C port (oracle/hmpc_port.c) driven by a memory-safety
  self-test at N = 1..60, both variants, mixed contact schedules, an
  infeasible start and B = 0 (tests/native/port_selftest.c, `make -C oracle
  sanitize`);
* the C ABI's argument validation (include/hmpc.h; hmpc_capi.cpp and the
  dispatch compiled with -fsanitize after -Xarch_host, the kernel objects
  linked as built), tests/native/capi_args.cpp -- every invalid call rejected
  before any launch (no GPU is needed; on a GPU host the live-context checks
  run too).

GPU code is not sanitized (no device ASan on this pool)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SAN = os.path.join(ROOT, 'oracle', '_san')
ENV = dict(os.environ, ASAN_OPTIONS='detect_leaks=0:abort_on_error=0', UBSAN_OPTIONS='print_stacktrace=1')


def _check(cmd):
    r = subprocess.run(cmd, capture_output=True, text=True, env=ENV, timeout=600)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-4000:]
    assert 'AddressSanitizer' not in out and 'runtime error' not in out, out[-4000:]
    return out


def test_port_under_asan_ubsan():
    subprocess.check_call(['make', '-s', '-C', os.path.join(ROOT, 'oracle'), 'sanitize'])
    out = _check([os.path.join(SAN, 'port_selftest')])
    assert 'variant 3 N 60' in out


@pytest.mark.skipif(shutil.which('/opt/rocm/bin/hipcc') is None, reason='hipcc absent')
def test_capi_argument_checks_under_asan_ubsan(tmp_path):
    pkg = os.path.join(ROOT, 'hopper-mpc-inertial_amd')
    # build.sh writes the kernel objects it linked into libhmpc.so (everything but the
    # ABI and dispatch host code, rebuilt below under the sanitizers)
    listing = os.path.join(pkg, 'build', 'objs.txt')

    def _objs():
        if not os.path.exists(listing):
            return None
        with open(listing) as f:
            objs = [os.path.join(pkg, p) for p in f.read().split()]
        return objs if objs and all(os.path.exists(o) for o in objs) else None

    objs = _objs()
    if objs is None:
        subprocess.check_call(['bash', os.path.join(pkg, 'build.sh')])
        objs = _objs()
    assert objs, 'build.sh wrote no object list'
    hip = '/opt/rocm/bin/hipcc'
    san = ['-Xarch_host', '-fsanitize=address', '-Xarch_host', '-fsanitize=undefined']
    flags = ['--offload-arch=gfx950', '-O1', '-g', '-std=c++17'] + san
    mine = []
    for src in (os.path.join(ROOT, 'tests', 'native', 'capi_args.cpp'),
                os.path.join(pkg, 'csrc', 'hmpc_capi.cpp'), os.path.join(pkg, 'csrc', 'hmpc_dispatch.cpp')):
        o = str(tmp_path / (os.path.basename(src) + '.o'))
        subprocess.check_call([hip] + flags + ['-c', src, '-o', o])
        mine.append(o)
    exe = str(tmp_path / 'capi_args')
    subprocess.check_call([hip, '--offload-arch=gfx950'] + san + mine + objs + ['-o', exe])
    out = _check([exe])
    assert 'capi_args: 0 failure(s)' in out
