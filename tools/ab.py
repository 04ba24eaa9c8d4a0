#!/usr/bin/env python3
"""Interleaved A/B of libhmpc builds on one bench workload (GPU box).

    python tools/ab.py --tag NAME --rounds 2 --args "--N 10" lib_a.so lib_b.so ...
    python tools/ab.py --tag NAME --args "--N 60" --vary "--order index" --vary "--order longest_first"

Each round runs ``bench.py <args> --cpu-seconds 0`` once per library
(HMPC_LIB=<lib>, each run under its own time limit) -- or, with --vary, once
per extra-argument set on libhmpc.so -- in order, so clock and
thermal drift spread over every variant.  Writes gpurun_out/ab/<tag>.json
(every line) and prints a table of the median solves/s and kernel ms per
library.  Stops at the first failing run (no retries on the GPU).
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--tag', required=True)
    ap.add_argument('--rounds', type=int, default=2)
    ap.add_argument('--args', default='')
    ap.add_argument('--timeout', type=int, default=240)
    ap.add_argument('--vary', action='append', default=[],
                    help='extra bench arguments of one variant (repeat; the library is libhmpc.so)')
    ap.add_argument('libs', nargs='*')
    a = ap.parse_args()
    # (library, extra arguments, label) per variant
    if a.vary:
        variants = [('libhmpc.so', v.split(), v) for v in a.vary]
    else:
        variants = [(lib, [], lib) for lib in a.libs]
    out = os.path.join(ROOT, 'gpurun_out', 'ab')
    os.makedirs(out, exist_ok=True)
    res = {lab: [] for _, _, lab in variants}
    for r in range(a.rounds):
        for lib, extra, lab in variants:
            # "libhmpc.so:NAME=VALUE,..." runs the library with those environment variables
            libname, _, envs = lib.partition(':')
            path = libname if os.path.isabs(libname) else os.path.join(ROOT, 'hopper-mpc-inertial_amd', libname)
            env = dict(os.environ, HMPC_LIB=path)
            for kv in filter(None, envs.split(',')):
                k, _, v = kv.partition('=')
                env[k] = v
            cmd = ['timeout', '-k', '10', str(a.timeout), sys.executable, os.path.join(ROOT, 'bench.py'),
                   '--cpu-seconds', '0'] + a.args.split() + extra
            p = subprocess.run(cmd, env=env, capture_output=True, text=True, cwd=ROOT)
            if p.returncode != 0:
                print(f'{lab} round {r}: rc {p.returncode}\n{p.stderr[-3000:]}', flush=True)
                json.dump(res, open(os.path.join(out, f'{a.tag}.json'), 'w'), indent=1)
                sys.exit(1)
            line = json.loads(p.stdout.strip().splitlines()[-1])
            res[lab].append(line)
            print(f'{a.tag} r{r} {lab}: {line["value"] / 1e6:.3f} M/s kernel {line["roofline"]["kernel_ms"]:.4f} ms '
                  f'{line["roofline"]["kernel"]}', flush=True)
    json.dump(res, open(os.path.join(out, f'{a.tag}.json'), 'w'), indent=1)
    print(f'== {a.tag} ({a.args}): median over {a.rounds} rounds')
    for lib, lines in res.items():
        v = statistics.median(x['value'] for x in lines) / 1e6
        k = statistics.median(x['roofline']['kernel_ms'] for x in lines)
        print(f'  {lib:28s} {v:8.3f} M/s  kernel {k:.4f} ms')


if __name__ == '__main__':
    main()
