"""Copy the judged profile evidence of tools/profile_r02.sh into profiles/.

    python tools/summarize_r02.py r02 [cfg ...]

For each configuration (gpurun_out/<tag>/<cfg>/) writes
  profiles/<tag>_<cfg>_bench.json        the bench line of that call
  profiles/<tag>_<cfg>_kernel_stats.csv  rocprofv3 --kernel-trace --stats summary
  profiles/<tag>_<cfg>_pmc.json          per-dispatch PMC means of the solve kernel
and updates profiles/traffic.json (read by bench.py): HBM bytes per launch =
2 x FETCH_SIZE + WRITE_SIZE (MI355X_MICROARCH.md: FETCH_SIZE reports half
the bytes of wide streaming reads; the raw sum is kept beside it) and the
executed fp64 flops per solve (64 lanes x (2 FMA + MUL + ADD + TRANS) wave
instructions / instances).
"""
import collections
import csv
import glob
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def kernel_token(name):
    """'hmpc::ric_kernel<3>' -> 'ric_kernel<3>' (matches the demangled
    rocprof name without matching ric_overflow_kernel)."""
    return name.split('::')[-1].replace(' ', '')


def pmc(cfgdir, token):
    agg = collections.defaultdict(list)
    for f in glob.glob(os.path.join(cfgdir, 'pmc_*', '*', 'run_counter_collection.csv')) + \
            glob.glob(os.path.join(cfgdir, 'pmc_*', 'run_counter_collection.csv')):
        per = collections.defaultdict(float)
        for r in csv.DictReader(open(f)):
            if token not in r['Kernel_Name'].replace(' ', ''):
                continue
            per[(r['Dispatch_Id'], r['Counter_Name'])] += float(r['Counter_Value'])
        for (_, c), v in per.items():
            agg[c].append(v)
    return {c: sum(v) / len(v) for c, v in agg.items()}


def main(tag, cfgs):
    dst = os.path.join(ROOT, 'profiles')
    tpath = os.path.join(dst, 'traffic.json')
    tj = json.load(open(tpath)) if os.path.exists(tpath) else {}
    for cfg in cfgs:
        src = os.path.join(ROOT, 'gpurun_out', tag, cfg)
        bench = json.loads(open(os.path.join(src, 'bench.json')).read().strip().splitlines()[-1])
        json.dump(bench, open(os.path.join(dst, f'{tag}_{cfg}_bench.json'), 'w'), indent=1)
        stats = glob.glob(os.path.join(src, 'trace', '**', 'run_kernel_stats.csv'), recursive=True)
        if stats:
            shutil.copy(stats[0], os.path.join(dst, f'{tag}_{cfg}_kernel_stats.csv'))
        kernel = bench['roofline']['kernel']
        B = bench['roofline']['solves_per_launch']
        m = pmc(src, kernel_token(kernel))
        waves = m.get('SQ_WAVES', 0.0) or 1.0
        f64 = 64 * (2 * m.get('SQ_INSTS_VALU_FMA_F64', 0) + m.get('SQ_INSTS_VALU_MUL_F64', 0) +
                    m.get('SQ_INSTS_VALU_ADD_F64', 0) + m.get('SQ_INSTS_VALU_TRANS_F64', 0))
        summary = {'kernel': kernel, 'instances_per_launch': B, 'waves_per_launch': waves,
                   'counters_per_dispatch': m,
                   'per_instance': {k: v / B for k, v in m.items() if k.startswith('SQ_INSTS')},
                   'fp64_flops_executed_per_solve': f64 / B,
                   'note': 'SQ_* are wave-level counts summed over the launch; per_instance divides by '
                           'the instances per launch (dense kernel: one wave per instance; Riccati '
                           'kernel: persistent waves, several instances each)'}
        if 'SQ_WAVE_CYCLES' in m:
            summary['wait_any_frac'] = m.get('SQ_WAIT_ANY', 0) / m['SQ_WAVE_CYCLES']
            summary['valu_active_frac'] = m.get('SQ_ACTIVE_INST_VALU', 0) / m['SQ_WAVE_CYCLES']
        if 'TCC_HIT_sum' in m:
            summary['l2_hit_rate'] = m['TCC_HIT_sum'] / max(1.0, m['TCC_HIT_sum'] + m['TCC_MISS_sum'])
        if 'GRBM_GUI_ACTIVE' in m:
            summary['grbm_gui_active'] = m['GRBM_GUI_ACTIVE']
        if 'FETCH_SIZE' in m and 'WRITE_SIZE' in m:
            fetch, write = 1024.0 * m['FETCH_SIZE'], 1024.0 * m['WRITE_SIZE']
            alg = bench['roofline']['algorithmic_bytes_per_solve'] * B
            summary['hbm_bytes_per_launch'] = {'fetch_raw': fetch, 'write': write, 'raw_total': fetch + write,
                                               'x2_corrected_total': 2 * fetch + write,
                                               'algorithmic': alg,
                                               'x2_corrected_over_algorithmic': (2 * fetch + write) / alg}
            c = bench['config']
            wl = f"{c['variant']}_N{c['horizon']}_B{B}_{c['plan']}{'_musweep' if c['mu_sweep'] else ''}" \
                 f"{'' if c['precision'] == 'f64' else '_' + c['precision']}"
            tj[wl] = {'kernel': kernel, 'bytes_per_launch_x2_corrected': 2 * fetch + write,
                      'bytes_per_launch_raw': fetch + write, 'fetch_bytes_raw': fetch, 'write_bytes': write,
                      'fp64_flops_executed_per_solve': f64 / B,
                      'source': f'profiles/{tag}_{cfg}_pmc.json (rocprofv3 --pmc FETCH_SIZE, WRITE_SIZE, '
                                f'SQ_INSTS_VALU_*_F64)'}
        json.dump(summary, open(os.path.join(dst, f'{tag}_{cfg}_pmc.json'), 'w'), indent=1)
        print(cfg, kernel, json.dumps({k: summary.get(k) for k in ('wait_any_frac', 'valu_active_frac',
                                                                 'l2_hit_rate', 'fp64_flops_executed_per_solve')}),
              summary.get('hbm_bytes_per_launch', {}).get('x2_corrected_over_algorithmic'))
    json.dump(tj, open(tpath, 'w'), indent=1)


if __name__ == '__main__':
    main(sys.argv[1], sys.argv[2:] or ['n10', 'n20', 'n60', 'n10_2f'])
