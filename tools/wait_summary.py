"""Summarise tools/wait_pmc.sh: what the waves of one kernel wait on.

    python tools/wait_summary.py <tag> <name> <kernel substring> [out.json]

Per wave of the kernel (sums over the PMC run's dispatches / SQ_WAVES):
  cycles            SQ_WAVE_CYCLES x 4 (quad-cycles -> cycles)
  wait_any          SQ_WAIT_ANY x 4: parked on s_waitcnt / barrier
  wait_inst_any     SQ_WAIT_INST_ANY x 4: issue stalls
  vmem / lds / smem in flight: derived latency x instructions = cycles in
      which an instruction of that kind was outstanding (they overlap each
      other and the issue; a wave parked on s_waitcnt waits on at least one)
and the vector-L1 / L2 side of the VMEM stream (TCP read requests to L2 and
their mean latency, L2 hit rate, HBM read requests).
"""
import collections
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def load(d, sub):
    """{counter: (sum over matching dispatches, dispatch count)}"""
    acc = collections.defaultdict(lambda: [0.0, 0])
    for f in glob.glob(os.path.join(d, 'pmc_*', '**', '*counter_collection.csv'), recursive=True):
        for r in csv.DictReader(open(f)):
            if sub not in r['Kernel_Name']:
                continue
            a = acc[r['Counter_Name']]
            a[0] += float(r['Counter_Value'])
            a[1] += 1
    return acc


def main(tag, name, sub, out=None):
    d = os.path.join(ROOT, 'gpurun_out', tag, name)
    acc = load(d, sub)
    tot = {k: v[0] for k, v in acc.items()}
    mean = {k: v[0] / max(v[1], 1) for k, v in acc.items()}   # the derived latencies: per dispatch
    waves = tot['SQ_WAVES']
    per_wave = lambda c: 4.0 * tot[c] / waves  # noqa: E731  (quad-cycles)
    res = {'kernel_match': sub, 'waves': waves,
           'cycles_per_wave': per_wave('SQ_WAVE_CYCLES'),
           'wait_any_per_wave': per_wave('SQ_WAIT_ANY'),
           'wait_inst_any_per_wave': per_wave('SQ_WAIT_INST_ANY'),
           'active_valu_per_wave': per_wave('SQ_ACTIVE_INST_VALU'),
           'active_lds_per_wave': per_wave('SQ_ACTIVE_INST_LDS'),
           'active_vmem_per_wave': per_wave('SQ_ACTIVE_INST_VMEM'),
           'active_salu_per_wave': per_wave('SQ_ACTIVE_INST_SCA'),
           'wait_inst_lds_per_wave': per_wave('SQ_WAIT_INST_LDS'),
           'insts_per_wave': {c: tot[c] / waves for c in ('SQ_INSTS_VMEM', 'SQ_INSTS_VMEM_RD', 'SQ_INSTS_VMEM_WR',
                                                            'SQ_INSTS_LDS', 'SQ_INSTS_SMEM_NORM') if c in tot},
           'latency_cycles': {c: mean[c] for c in ('VmemLatency', 'LdsLatency', 'SmemLatency') if c in mean}}
    lat = res['latency_cycles']
    ins = res['insts_per_wave']
    res['in_flight_cycles_per_wave'] = {
        'vmem': lat.get('VmemLatency', 0) * ins.get('SQ_INSTS_VMEM', 0),
        'lds': lat.get('LdsLatency', 0) * ins.get('SQ_INSTS_LDS', 0),
        'smem': lat.get('SmemLatency', 0) * ins.get('SQ_INSTS_SMEM_NORM', 0)}
    if 'TCP_TCC_READ_REQ_sum' in tot:
        res['tcp_to_l2_reads_per_wave'] = tot['TCP_TCC_READ_REQ_sum'] / waves
        res['tcp_to_l2_read_latency'] = tot.get('TCP_TCC_READ_REQ_LATENCY_sum', 0) / max(1.0, tot['TCP_TCC_READ_REQ_sum'])
        res['tcp_cache_accesses_per_wave'] = tot.get('TCP_TOTAL_CACHE_ACCESSES_sum', 0) / waves
        res['tcp_pending_stall_per_wave'] = tot.get('TCP_PENDING_STALL_CYCLES_sum', 0) / waves
    if 'TCC_HIT_sum' in tot:
        res['l2_hit_rate'] = tot['TCC_HIT_sum'] / max(1.0, tot['TCC_HIT_sum'] + tot['TCC_MISS_sum'])
        res['l2_to_fabric_reads_per_wave'] = tot.get('TCC_EA0_RDREQ_sum', 0) / waves
        res['l2_to_dram_reads_per_wave'] = tot.get('TCC_EA0_RDREQ_DRAM_sum', 0) / waves
    if 'TA_BUSY_sum' in tot:
        res['ta_busy_per_wave'] = tot['TA_BUSY_sum'] / waves
        res['ta_addr_stalled_by_tc_per_wave'] = tot.get('TA_ADDR_STALLED_BY_TC_CYCLES_sum', 0) / waves
    res['lds_bank_conflict_frac'] = tot.get('SQ_LDS_BANK_CONFLICT', 0) / max(1.0, tot.get('SQ_LDS_IDX_ACTIVE', 1))
    print(json.dumps(res, indent=1))
    if out:
        json.dump(res, open(out, 'w'), indent=1)


if __name__ == '__main__':
    main(*sys.argv[1:])
