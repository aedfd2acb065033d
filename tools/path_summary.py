"""Summarise tools/profile_round.sh output into one JSON per path (profiles/pmc_<path>.json): per kernel the rocprofv3
kernel-trace duration, launches per step, HBM bytes per launch from the FETCH_SIZE / WRITE_SIZE passes (gfx950
correction per MI355X_MICROARCH.md: FETCH_SIZE counts half of a wide stream, so reads are doubled), achieved GB/s,
and the kernel's I/O-contract bytes where the layout fixes them (tiles it must write or read once, slabs, params),
so traffic / io_bytes > 1 shows re-reads; per path the totals per step and the MFMA fraction of the path's
algorithmic flops (SURVEY.md §8a work units).

usage: python tools/path_summary.py <round dir> <out dir>   (round dir holds <path>/{timing.json, trace, pmc1, pmc2})
"""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from profile_paths import PATHS, flop_per_coord  # noqa: E402

PEAK_TF, HBM_GBS = 157.3, 8000.


def short(name):
    m = re.match(r'(?:void )?siren::(?:\(anonymous namespace\)::)?(\w+)(<[^(]*>)?', name)
    if not m:
        return name[:60]
    return m.group(1) + (m.group(2).replace(' ', '') if m.group(2) else '')


def plan(path):
    """Split-K plan of the W2-style backward (siren_capi.hip TrainPlan / JetPlan): (n_pad, columns, S, P)."""
    d, H, L, o, n, _ = PATHS[path]
    jet = path.startswith('poisson')
    P = H * d + H + L * (H * H + H) + o * H + o
    if path == 'hypernet':
        n = 4096
    n_pad = (n + (15 if jet else 63)) // (16 if jet else 64) * (16 if jet else 64)
    # jet paths: 4 streams per coordinate; w3_wide: the two-stream (value, tangent) tiles of the hidden-512 W3
    cols = 4 * n_pad if jet else (2 * n_pad if path == 'w3_wide' else n_pad)
    tiles = cols // 16
    want = max(1, 256 // (L * (H // 256) ** 2))
    if path == 'hypernet':
        want = max(1, 512 // (L * (H // 256) ** 2) // 32)
    S = max(1, min(tiles, want))
    tps = max(1, -(-tiles // S))
    S = max(1, -(-tiles // tps))
    return n_pad, cols, S, P


def io_bytes(path, k):
    """Bytes the kernel must move by its I/O contract (None where the layout does not fix a simple figure)."""
    d, H, L, o, n, _ = PATHS[path]
    n_pad, cols, S, P = plan(path)
    B = 32 if path == 'hypernet' else 1
    T = H * 4  # one layer's tile bytes per column
    hid = L * (H * H + H)
    if k.startswith('wgrad_kernel'):   # a_{l-1} and delta_l tiles of the hidden layers, S hidden-layer slabs
        per = 2 * L * cols * T + S * hid * 4   # (w3_theta / sdf: one of the two launches, (A, D) or (At, Dt))
        return B * per
    if k.startswith('edge_kernel'):    # delta_0 / a_L rows + the coordinate scalars, S edge slabs
        return B * (2 * cols * T + S * (P - hid) * 4) if path not in ('w3_theta', 'sdf') else None
    if k.startswith('reduce_kernel'):  # the slabs once, the gradient once
        return B * (S * P * 4 + P * 4) if path not in ('w3_theta', 'sdf') else None
    if k.startswith('jet_store_kernel<1'):   # JET_FWD: a-jets + z-jets of L + 1 layers written, x read, outputs
        return 2 * (L + 1) * cols * T + n * (d + 1) * 4
    if k.startswith('jet_store_kernel<2'):   # JET_REV: z-jets read, zb-jets written
        return 2 * (L + 1) * cols * T
    if k.startswith('hess_kernel<true'):  # the Hessian node's forward: x read, the kept 6-stream jets and Hm written
        return 6 * (L + 1) * n_pad * T + n * (d + d * d) * 4
    if k.startswith('hess_kernel'):
        return n * (d + d * d) * 4
    if k.startswith('jet_store_kernel<0,true,true,true'):  # reverse-only QG jet: kept jets read, a- and zb-jets written
        return 6 * (L + 1) * n_pad * T + 2 * (L + 1) * cols * T + n * (d + d * d) * 4
    if k.startswith('jet_store_kernel<0,true'):  # mixed jet (both phases): a-, z-, zb-jets
        return 3 * (L + 1) * cols * T + n * 3 * d * 4
    if k.startswith('lay_'):  # layered path epilogues, per 16384-coordinate chunk (layered.hip)
        C, tile = min(n, 16384), min(n, 16384) * H * 4
        return {'lay_first_kernel': 2 * tile + C * d * 4, 'lay_sine_kernel': 3 * tile,
                'lay_last_kernel': 3 * tile + C * o * 4, 'lay_rev_kernel<0>': 3 * tile,
                'lay_rev_kernel<1>': 3 * tile + C * o * 4, 'lay_rev_kernel<2>': 3 * tile + C * d * 4}.get(k)
    # (hypernet: n_pad is one element's, n the whole batch; every element's weight stream is read once)
    stream = B * (2 * L * H * H * 4) if path == 'hypernet' else 0
    if re.match(r'w1_kernel<\d+,4>', k) or (k.startswith('wide_kernel<4') and path == 'video'):
        return B * 2 * (L + 1) * n_pad * T + n * (d + o) * 4 + stream // 2   # FWDS: a tiles + cos of L + 1 layers
    if re.match(r'w1_kernel<\d+,5>', k) or k.startswith('wide_kernel<5'):
        return B * ((L + 1) * n_pad * T + L * n_pad * T) + n * (d + o) * 4 + stream // 2  # REV: cos read, deltas
    return None


def trace_stats(d):
    out = {}
    for path in glob.glob(os.path.join(d, '**', '*kernel_stats.csv'), recursive=True):
        for row in csv.DictReader(open(path)):
            k = short(row['Name'])
            out[k] = {'calls': int(row['Calls']), 'avg_ns': float(row['AverageNs']),
                      'total_ns': float(row['TotalDurationNs'])}
    return out


def pmc(d):
    vals = defaultdict(lambda: defaultdict(list))
    for path in glob.glob(os.path.join(d, '**', '*counter_collection.csv'), recursive=True):
        for row in csv.DictReader(open(path)):
            vals[short(row['Kernel_Name'])][row['Counter_Name']].append(float(row['Counter_Value']))
    return {k: {c: sum(v) / len(v) for c, v in cs.items()} for k, cs in vals.items()}


def summarise(rdir, path):
    pdir = os.path.join(rdir, path)
    timing = json.load(open(os.path.join(pdir, 'timing.json')))
    steps = timing['steps_total']
    tr = trace_stats(os.path.join(pdir, 'trace'))
    cnt = pmc(pdir)
    d, H, L, o, n, units = PATHS[path]
    kernels, tot_ns, tot_bytes, tot_io = {}, 0., 0., 0.
    io_known = True
    for k, t in sorted(tr.items()):
        c = cnt.get(k, {})
        rd = 2 * 1024 * c.get('FETCH_SIZE', 0.)
        wr = 1024 * c.get('WRITE_SIZE', 0.)
        per_step = t['calls'] / steps
        io = io_bytes(path, k)
        rec = {'launches_per_step': round(per_step, 3), 'avg_us': round(t['avg_ns'] / 1e3, 2),
               'hbm_read_bytes_per_launch': round(rd), 'hbm_write_bytes_per_launch': round(wr),
               'hbm_gbs': round((rd + wr) / t['avg_ns'], 1) if t['avg_ns'] > 0 else None,
               'hbm_frac': round((rd + wr) / t['avg_ns'] / HBM_GBS, 4) if t['avg_ns'] > 0 else None,
               'io_bytes_per_launch': io, 'traffic_over_io': round((rd + wr) / io, 3) if io else None}
        if 'SQ_INSTS_MFMA' in c or 'SQ_WAVE_CYCLES' in c:
            # SQ counters (MI355X_MICROARCH.md: SQ_WAVE_CYCLES / SQ_WAIT_* / SQ_ACTIVE_INST_* in quad-cycles,
            # SQ_VALU_MFMA_BUSY_CYCLES in cycles summed over SIMDs; GRBM_GUI_ACTIVE summed over the 8 XCDs)
            rec['sq'] = {kk: c[kk] for kk in sorted(c) if kk.startswith('SQ_') or kk.startswith('GRBM')}
            mf = c.get('SQ_INSTS_MFMA', 0.)
            if mf:
                rec['valu_per_mfma'] = round(c.get('SQ_INSTS_VALU', 0.) / mf, 3)
                rec['lds_per_mfma'] = round(c.get('SQ_INSTS_LDS', 0.) / mf, 3) if 'SQ_INSTS_LDS' in c else None
            if c.get('GRBM_GUI_ACTIVE') and c.get('SQ_VALU_MFMA_BUSY_CYCLES'):
                rec['mfma_busy_frac'] = round(c['SQ_VALU_MFMA_BUSY_CYCLES'] / 1024 / (c['GRBM_GUI_ACTIVE'] / 8), 4)
            if c.get('SQ_WAVE_CYCLES'):
                rec['wait_inst_any_frac'] = round(c.get('SQ_WAIT_INST_ANY', 0.) / c['SQ_WAVE_CYCLES'], 4)
                rec['wait_any_frac'] = round(c.get('SQ_WAIT_ANY', 0.) / c['SQ_WAVE_CYCLES'], 4)
                rec['active_inst_any_frac'] = round(c.get('SQ_ACTIVE_INST_ANY', 0.) / c['SQ_WAVE_CYCLES'], 4)
            if c.get('SQ_INSTS_LDS'):
                rec['lds_bank_conflict_per_lds_inst'] = round(c.get('SQ_LDS_BANK_CONFLICT', 0.) / c['SQ_INSTS_LDS'], 4)
        kernels[k] = rec
        tot_ns += t['avg_ns'] * per_step
        tot_bytes += (rd + wr) * per_step
        if io is None and (rd + wr) > 1e6:
            io_known = False
        tot_io += (io or 0.) * per_step
    flops = units * flop_per_coord(d, H, L, o) * n
    return {'path': path, 'n': n, 'config': {'d_in': d, 'hidden': H, 'hidden_layers': L, 'd_out': o},
            'work_units_of_F': units, 'flop_per_step': flops, 'hip_event_ms_per_step': timing['ms_per_step'],
            'kernel_ms_per_step': round(tot_ns / 1e6, 4),
            'mfma_frac_of_kernel_time': round(flops / (tot_ns * 1e-9) / 1e12 / PEAK_TF, 4) if tot_ns else None,
            'hbm_bytes_per_step': round(tot_bytes), 'io_bytes_per_step': round(tot_io) if io_known else None,
            'kernels': kernels}


def main(rdir, outdir):
    for pdir in sorted(glob.glob(os.path.join(rdir, '*', 'timing.json'))):
        path = os.path.basename(os.path.dirname(pdir))
        res = summarise(rdir, path)
        with open(os.path.join(outdir, 'pmc_%s.json' % path), 'w') as f:
            json.dump(res, f, indent=1, sort_keys=True)
        print('%-12s %8.3f ms/step kernels %8.3f ms  mfma %.3f  hbm %.1f MB/step' % (
            path, res['hip_event_ms_per_step'], res['kernel_ms_per_step'], res['mfma_frac_of_kernel_time'] or 0,
            res['hbm_bytes_per_step'] / 1e6))
        for k, v in res['kernels'].items():
            print('    %-34s x%-5g %9.2f us  %8.1f GB/s  io x%s' % (k, v['launches_per_step'], v['avg_us'],
                                                                v['hbm_gbs'] or 0, v['traffic_over_io']))


if __name__ == '__main__':
    main(sys.argv[1], sys.argv[2])
