"""Summarise rocprofv3 --pmc CSV passes (tools/run_pmc.sh) into per-kernel per-dispatch averages (JSON).

HBM bytes follow MI355X_MICROARCH.md §HBM: FETCH_SIZE (KiB) reads exactly half of a wide coalesced stream on
gfx950, so reads are doubled; WRITE_SIZE (KiB) is exact for 16-B-per-lane stores (ours are 4-16 B: noted).
usage: python tools/pmc_summary.py <pmc dir> <n coords> <out.json>
"""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict


def short(name):
    m = re.match(r'(?:void )?siren::(\w+)(<[^>]*>)?', name)
    if not m:
        return name[:60]
    return m.group(1) + (m.group(2).replace(' ', '') if m.group(2) else '')


def main(d, n, out):
    vals = defaultdict(lambda: defaultdict(list))
    dur = defaultdict(list)
    for path in glob.glob(os.path.join(d, 'pass*', '*counter_collection.csv')):
        for row in csv.DictReader(open(path)):
            k = short(row['Kernel_Name'])
            vals[k][row['Counter_Name']].append(float(row['Counter_Value']))
            dur[k].append((int(row['End_Timestamp']) - int(row['Start_Timestamp'])) * 1e-9)
    res = {}
    for k, cs in vals.items():
        avg = {c: sum(v) / len(v) for c, v in cs.items()}
        r = {'counters_avg_per_dispatch': avg, 'profiled_duration_s_avg': sum(dur[k]) / len(dur[k])}
        if 'FETCH_SIZE' in avg or 'WRITE_SIZE' in avg:
            rd = 2 * 1024 * avg.get('FETCH_SIZE', 0.)   # gfx950: FETCH_SIZE counts half of a wide stream
            wr = 1024 * avg.get('WRITE_SIZE', 0.)
            r['hbm_read_bytes_per_launch'] = rd
            r['hbm_write_bytes_per_launch'] = wr
            r['hbm_bytes_per_launch'] = rd + wr
        if 'SQ_WAVE_CYCLES' in avg and avg['SQ_WAVE_CYCLES'] > 0:
            w = avg['SQ_WAVE_CYCLES']
            r['wait_any_frac'] = avg.get('SQ_WAIT_ANY', 0) / w
            r['wait_inst_any_frac'] = avg.get('SQ_WAIT_INST_ANY', 0) / w
            r['active_inst_any_frac'] = avg.get('SQ_ACTIVE_INST_ANY', 0) / w
        if 'GRBM_GUI_ACTIVE' in avg:
            r['effective_clock_ghz'] = avg['GRBM_GUI_ACTIVE'] / 8 / r['profiled_duration_s_avg'] / 1e9
        if 'SQ_VALU_MFMA_BUSY_CYCLES' in avg and 'GRBM_GUI_ACTIVE' in vals[k]:
            pass
        res[k] = r
    # stamp: the sources of the library the profiled process ran (bench.py reports traffic only for a matching build)
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import __graft_entry__
    json.dump({'n': n, 'kernels': res, 'source_hash': __graft_entry__._source_hash()}, open(out, 'w'), indent=1,
              sort_keys=True)
    print(json.dumps({k: {kk: vv for kk, vv in v.items() if kk != 'counters_avg_per_dispatch'} for k, v in res.items()},
                     indent=1))
    for k, v in res.items():
        print(k, {c: '%.4g' % x for c, x in v['counters_avg_per_dispatch'].items()})


if __name__ == '__main__':
    main(sys.argv[1], int(sys.argv[2]), sys.argv[3])
