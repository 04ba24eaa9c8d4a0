"""Copy the judged profile evidence of one GPU call into profiles/.

    python tools/summarize_profiles.py r01

reads gpurun_out/<tag>/ (bench.json, trace/run_kernel_stats.csv) and
gpurun_out/pmc_<tag>/ (rocprofv3 --pmc passes) and writes
  profiles/<tag>_bench.json           the bench line of that call
  profiles/<tag>_kernel_stats.csv     rocprofv3 --kernel-trace --stats summary
  profiles/<tag>_pmc_summary.json     per-dispatch PMC means of the solve kernel
  profiles/traffic.json               HBM bytes per launch (read by bench.py)
HBM bytes = FETCH_SIZE + WRITE_SIZE (KiB units in rocprofv3).  Per
MI355X_MICROARCH.md, FETCH_SIZE reports half the bytes of 16-B-per-lane
streaming reads; this kernel reads 8 B per lane (uncalibrated), so the raw
sum is recorded together with the 2x-corrected read figure.
"""
import collections
import csv
import glob
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def pmc(tag):
    agg = collections.defaultdict(list)
    for f in glob.glob(os.path.join(ROOT, 'gpurun_out', f'pmc_{tag}', '*', 'run_counter_collection.csv')):
        per = collections.defaultdict(float)
        for r in csv.DictReader(open(f)):
            if 'solve_kernel' not in r['Kernel_Name']:
                continue
            per[(r['Dispatch_Id'], r['Counter_Name'])] += float(r['Counter_Value'])
        for (_, c), v in per.items():
            agg[c].append(v)
    return {c: sum(v) / len(v) for c, v in agg.items()}


def main(tag):
    src = os.path.join(ROOT, 'gpurun_out', tag)
    dst = os.path.join(ROOT, 'profiles')
    os.makedirs(dst, exist_ok=True)
    bench = json.loads(open(os.path.join(src, 'bench.json')).read().strip().splitlines()[-1])
    json.dump(bench, open(os.path.join(dst, f'{tag}_bench.json'), 'w'), indent=1)
    shutil.copy(os.path.join(src, 'trace', 'run_kernel_stats.csv'),
                os.path.join(dst, f'{tag}_kernel_stats.csv'))
    m = pmc(tag)
    waves = m.get('SQ_WAVES', 0.0) or 1.0
    summary = {'counters_per_dispatch': m,
               'per_instance': {k: v / waves for k, v in m.items() if k.startswith('SQ_INSTS')},
               'note': 'SQ_* are wave-level counts; one wave (N=10) = one QP instance'}
    if 'FETCH_SIZE' in m and 'WRITE_SIZE' in m:
        fetch, write = 1024.0 * m['FETCH_SIZE'], 1024.0 * m['WRITE_SIZE']
        summary['hbm_bytes_per_launch'] = {'fetch_raw': fetch, 'write': write,
                                           'raw_total': fetch + write,
                                           'fetch_x2_corrected_total': 2 * fetch + write}
        cfg = bench['config']
        wl = f"{cfg['variant']}_N{cfg['horizon']}_B{bench['roofline']['solves_per_launch']}_curve"
        tj_path = os.path.join(dst, 'traffic.json')
        tj = json.load(open(tj_path)) if os.path.exists(tj_path) else {}
        tj[wl] = {'bytes_per_launch': fetch + write, 'fetch_bytes': fetch, 'write_bytes': write,
                  'source': f'profiles/{tag}_pmc_summary.json (rocprofv3 --pmc FETCH_SIZE, WRITE_SIZE)'}
        if 'SQ_INSTS_VALU_FMA_F64' in m:
            # executed fp64 flops per solve: wave instructions x 64 lanes
            # (FMA = 2 flops; masked lanes included, so an upper bound)
            fl = 64.0 * (2 * m['SQ_INSTS_VALU_FMA_F64'] + m.get('SQ_INSTS_VALU_MUL_F64', 0.0)
                         + m.get('SQ_INSTS_VALU_ADD_F64', 0.0)) / waves
            tj[wl]['fp64_flops_per_solve'] = fl
            summary['fp64_flops_per_solve'] = fl
        json.dump(tj, open(tj_path, 'w'), indent=1)
    json.dump(summary, open(os.path.join(dst, f'{tag}_pmc_summary.json'), 'w'), indent=1)
    print(json.dumps(summary, indent=1))


if __name__ == '__main__':
    main(sys.argv[1] if len(sys.argv) > 1 else 'r01')
