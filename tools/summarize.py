"""Copy the judged profile evidence of tools/profile.sh into profiles/.

    python tools/summarize.py r04 [cfg ...]

For each configuration (gpurun_out/<tag>/<cfg>/) writes
  profiles/<tag>_<cfg>_bench.json        the bench line of that call
  profiles/<tag>_<cfg>_kernel_stats.csv  rocprofv3 --kernel-trace --stats summary
  profiles/<tag>_<cfg>_pmc.json          PMC counters per solve step
and updates profiles/traffic.json (read by bench.py).

A solve step may be several kernels (the dense split launch: classify, the
compacted and the full kernel; every solve: the overflow pass), so counters
are summed over every hmpc:: dispatch of the PMC run and divided by the
number of steps (dispatches of the step's main kernel).  Derived figures:
  HBM bytes per step = 2 x FETCH_SIZE + WRITE_SIZE (x1024 B; FETCH_SIZE
      reports half the bytes of wide streaming reads on gfx950,
      MI355X_MICROARCH.md; the raw sum is kept beside it)
  executed fp64 flops per solve = 64 lanes x (2 FMA + MUL + ADD + TRANS) wave
      instructions / instances
  valu_busy = SQ_ACTIVE_INST_VALU x 4 / (1024 SIMDs x GRBM_GUI_ACTIVE / 8):
      SQ_ACTIVE_INST_VALU counts quad-cycles summed over waves, GRBM_GUI_ACTIVE
      cycles summed over the 8 XCDs (PMC collection serialises the kernels)
  resident waves / SIMD = SQ_WAVE_CYCLES x 4 / (1024 x GRBM_GUI_ACTIVE / 8)
"""
import collections
import csv
import glob
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SIMDS = 1024
XCDS = 8


def tokens(kernel):
    """'hmpc::a<..> + hmpc::b<..>' -> ['a<..>', 'b<..>'] (demangled rocprof
    names without the namespace; spaces dropped)."""
    return [k.split('::')[-1].replace(' ', '') for k in kernel.split(' + ')]


def pmc(cfgdir, main_token):
    """Counters per step: sums over every hmpc:: dispatch / main-kernel dispatches."""
    tot = collections.defaultdict(float)
    steps = collections.defaultdict(set)
    per_kernel = collections.defaultdict(lambda: collections.defaultdict(float))
    files = glob.glob(os.path.join(cfgdir, 'pmc_*', '**', 'run_counter_collection.csv'), recursive=True)
    for f in files:
        for r in csv.DictReader(open(f)):
            name = r['Kernel_Name'].replace(' ', '')
            if 'hmpc::' not in name:
                continue
            c, v = r['Counter_Name'], float(r['Counter_Value'])
            tot[(f, c)] += v
            per_kernel[name.replace('(anonymousnamespace)::', '').split('(')[0]][c] += v
            if main_token in name:
                steps[f].add(r['Dispatch_Id'])
    out = {}
    for (f, c), v in tot.items():
        n = len(steps[f]) or 1
        out[c] = out.get(c, 0.0) + v / n
    nsteps = {f: len(s) for f, s in steps.items()}
    return out, nsteps, {k: dict(v) for k, v in per_kernel.items()}


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
        toks = tokens(kernel)
        m, nsteps, per_kernel = pmc(src, toks[-1])
        f64 = 64 * (2 * m.get('SQ_INSTS_VALU_FMA_F64', 0) + m.get('SQ_INSTS_VALU_MUL_F64', 0) +
                    m.get('SQ_INSTS_VALU_ADD_F64', 0) + m.get('SQ_INSTS_VALU_TRANS_F64', 0))
        summary = {'kernel': kernel, 'instances_per_step': B, 'counters_per_step': m,
                   'steps_per_pass': nsteps,
                   'per_instance': {k: v / B for k, v in m.items() if k.startswith('SQ_INSTS')},
                   'fp64_flops_executed_per_solve': f64 / B,
                   'counters_by_kernel_summed_over_the_run': per_kernel,
                   'note': 'counters summed over every hmpc:: dispatch of the PMC run, divided by the '
                           'steps (dispatches of the main kernel); SQ_* are wave-level sums'}
        cyc = m.get('GRBM_GUI_ACTIVE', 0.0) / XCDS
        if 'SQ_WAVE_CYCLES' in m:
            summary['wait_any_frac'] = m.get('SQ_WAIT_ANY', 0) / m['SQ_WAVE_CYCLES']
            summary['valu_active_frac_of_wave_cycles'] = m.get('SQ_ACTIVE_INST_VALU', 0) / m['SQ_WAVE_CYCLES']
        if cyc > 0:
            summary['grbm_cycles_per_step'] = cyc
            if 'SQ_ACTIVE_INST_VALU' in m:
                summary['valu_busy'] = m['SQ_ACTIVE_INST_VALU'] * 4 / (SIMDS * cyc)
            if 'SQ_WAVE_CYCLES' in m:
                summary['resident_waves_per_simd'] = m['SQ_WAVE_CYCLES'] * 4 / (SIMDS * cyc)
        # per kernel (PMC collection serialises the dispatches, so each kernel's
        # GRBM_GUI_ACTIVE is its own duration): the split's classes one by one
        dk = {}
        for kn, kc in per_kernel.items():
            kcyc = kc.get('GRBM_GUI_ACTIVE', 0.0) / XCDS
            d = {}
            if kcyc > 0 and 'SQ_ACTIVE_INST_VALU' in kc:
                d['valu_busy'] = kc['SQ_ACTIVE_INST_VALU'] * 4 / (SIMDS * kcyc)
            if kcyc > 0 and 'SQ_WAVE_CYCLES' in kc:
                d['resident_waves_per_simd'] = kc['SQ_WAVE_CYCLES'] * 4 / (SIMDS * kcyc)
            if kc.get('SQ_WAVE_CYCLES'):
                d['wait_any_frac'] = kc.get('SQ_WAIT_ANY', 0) / kc['SQ_WAVE_CYCLES']
                d['wait_inst_any_frac'] = kc.get('SQ_WAIT_INST_ANY', 0) / kc['SQ_WAVE_CYCLES']
            if 'TCC_HIT_sum' in kc:
                d['l2_hit_rate'] = kc['TCC_HIT_sum'] / max(1.0, kc['TCC_HIT_sum'] + kc['TCC_MISS_sum'])
            if d:
                dk[kn] = d
        summary['derived_by_kernel'] = dk
        if 'TCC_HIT_sum' in m:
            summary['l2_hit_rate'] = m['TCC_HIT_sum'] / max(1.0, m['TCC_HIT_sum'] + m['TCC_MISS_sum'])
        entry = {'kernel': kernel, 'fp64_flops_executed_per_solve': f64 / B,
                 'valu_busy': summary.get('valu_busy'), 'wait_any_frac': summary.get('wait_any_frac'),
                 'valu_insts_per_solve': m.get('SQ_INSTS_VALU', 0) / B if 'SQ_INSTS_VALU' in m else None,
                 'source': f'profiles/{tag}_{cfg}_pmc.json (rocprofv3 --pmc; FETCH_SIZE, WRITE_SIZE, '
                           f'SQ_INSTS_VALU_*_F64, SQ_ACTIVE_INST_VALU, GRBM_GUI_ACTIVE)'}
        if 'FETCH_SIZE' in m and 'WRITE_SIZE' in m:
            fetch, write = 1024.0 * m['FETCH_SIZE'], 1024.0 * m['WRITE_SIZE']
            alg = bench['roofline']['algorithmic_bytes_per_solve'] * B
            summary['hbm_bytes_per_step'] = {'fetch_raw': fetch, 'write': write, 'raw_total': fetch + write,
                                             'x2_corrected_total': 2 * fetch + write, 'algorithmic': alg,
                                             'x2_corrected_over_algorithmic': (2 * fetch + write) / alg}
            entry.update({'bytes_per_launch_x2_corrected': 2 * fetch + write, 'bytes_per_launch_raw': fetch + write,
                          'fetch_bytes_raw': fetch, 'write_bytes': write})
        c = bench['config']
        wl = f"{c['variant']}_N{c['horizon']}_B{B}_{c['plan']}{'_musweep' if c['mu_sweep'] else ''}" \
             f"{'' if c['precision'] == 'f64' else '_' + c['precision']}"
        tj[wl] = entry
        json.dump(summary, open(os.path.join(dst, f'{tag}_{cfg}_pmc.json'), 'w'), indent=1)
        print(cfg, kernel, json.dumps({k: summary.get(k) for k in ('valu_busy', 'resident_waves_per_simd',
                                                                 'wait_any_frac', 'l2_hit_rate',
                                                                 'fp64_flops_executed_per_solve')}),
              summary.get('hbm_bytes_per_step', {}).get('x2_corrected_over_algorithmic'))
    json.dump(tj, open(tpath, 'w'), indent=1)


if __name__ == '__main__':
    main(sys.argv[1], sys.argv[2:] or ['n10', 'n20', 'n60', 'n10_2f', 'n10_f32', 'n10_f32r'])
