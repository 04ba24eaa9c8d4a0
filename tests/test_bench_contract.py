"""bench.py's JSON line (the driver's contract, BASELINE.json's metric) and
its algorithmic figures.  The CPU tests pin the closed forms of SURVEY.md 8d;
the GPU test runs one short bench and checks every field the driver and the
judge read (a subprocess, as the driver runs it)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def test_algorithmic_bytes_match_the_survey():
    # in 8 (28N + 25), out 8 (18N + 13) + 4
    for N, total in ((10, 3988), (20, 7668), (60, 22388)):
        assert bench.algorithmic_bytes(N) == 8 * (28 * N + 25) + 8 * (18 * N + 13) + 4 == total


def test_workload_labels_name_the_baseline_configs():
    class A:   # bench.parse() defaults, then per config
        variant, N, straight, mu_sweep, precision, refine, batch, global_batch = '3f', 10, False, False, 'f64', 5, 65536, 0
    a = A()
    assert bench.workload_label(a, 1).startswith('configs[2]')
    a.precision = 'f32'
    assert bench.workload_label(a, 1).startswith('configs[4]')
    a.precision, a.variant, a.straight, a.batch = 'f64', '2f', True, 4096
    assert bench.workload_label(a, 1).startswith('configs[1]')
    a.variant, a.N, a.mu_sweep, a.global_batch = '3f', 20, True, 262144
    assert bench.workload_label(a, 8).startswith('configs[3]') and 'strong' in bench.workload_label(a, 8)


@pytest.mark.gpu
def test_bench_line_contract():
    cmd = [sys.executable, os.path.join(ROOT, 'bench.py'), '--steps', '3', '--warmup', '1', '--prewarm-ms', '100',
           '--cpu-seconds', '1', '--batch', '4096']
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=110, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith('{')]
    assert len(lines) == 1, out.stdout
    d = json.loads(lines[0])
    for k in ('metric', 'value', 'unit', 'n_gpus', 'steps', 'warmup', 'ms_per_step', 'higher_is_better', 'scaling',
              'vs_baseline', 'dtype', 'data', 'config', 'roofline', 'cpu_baseline', 'prewarm_ms', 'prewarm_steps'):
        assert k in d, k
    assert d['metric'] == bench.METRIC and d['unit'] == 'QP solves/s' and d['value'] > 0
    assert (d['n_gpus'], d['steps'], d['warmup']) == (1, 3, 1)
    assert d['higher_is_better'] is True and d['scaling'] == 'weak' and d['vs_baseline'] is None
    assert d['dtype'] == 'f64' and d['config']['workload'].startswith('configs[2]')
    assert abs(d['value'] - 4096 / (d['ms_per_step'] * 1e-3)) <= 1e-6 * d['value']
    r = d['roofline']
    for k in ('bound', 'achieved', 'peak', 'unit', 'frac', 'traffic'):
        assert k in r, k
    assert r['bound'] == 'hbm' and r['unit'] == 'GB/s' and abs(r['frac'] - r['achieved'] / r['peak']) < 1e-12
    c = d['cpu_baseline']
    for k in ('value', 'unit', 'cores', 'kind', 'sample'):
        assert k in c, k
    assert c['kind'] == 'port' and c['value'] > 0
    assert d['prewarm_ms'] >= 100 and d['prewarm_steps'] > 0
    p = d['parity_sample']
    assert p['instances'] > 0 and p['max_abs_du_vs_port'] <= 1e-6 and p['status_mismatch_total'] == 0
