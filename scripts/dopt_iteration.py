#!/usr/bin/env python
"""Steady-state densityopt iteration from a rocprofv3 kernel trace: the
iterations are cut at the fused S-step kernel (one per iteration, the last
launch of the sim half), the last --iters of them are kept (graph replays
only: the eager warm-up and capture iterations come first), and every launch
between two S steps is counted -- kernels, device copies (__amd_rocclr_*),
busy time and wall span per iteration.

    python scripts/dopt_iteration.py <dir with *kernel_trace.csv> [--iters 200] [--marker dopt_sstep_kernel]
"""
import argparse
import csv
import glob
import os
from collections import OrderedDict


def short(name):
    n = name.replace('(anonymous namespace)::', '').replace('btn::gpu::', '')
    return n.split('(')[0].replace('void ', '')[:90]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('dir')
    ap.add_argument('--iters', type=int, default=200)
    ap.add_argument('--marker', default='dopt_sstep_kernel')
    a = ap.parse_args()
    rows = []
    for f in glob.glob(os.path.join(a.dir, '**', '*kernel_trace.csv'), recursive=True):
        rows += list(csv.DictReader(open(f)))
    rows.sort(key=lambda r: int(r['Start_Timestamp']))
    marks = [i for i, r in enumerate(rows) if a.marker in r['Kernel_Name']]
    if len(marks) < 3:
        raise SystemExit(f'{len(marks)} {a.marker} launches in the trace')
    marks = marks[-(a.iters + 1):]
    n = len(marks) - 1
    agg = OrderedDict()
    busy = span = 0.0
    copies = 0
    for k in range(n):
        it = rows[marks[k] + 1:marks[k + 1] + 1]
        t0, t1 = int(it[0]['Start_Timestamp']), int(it[-1]['End_Timestamp'])
        span += (t1 - t0) * 1e-3
        for r in it:
            d = (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) * 1e-3
            busy += d
            nm = short(r['Kernel_Name'])
            copies += nm.startswith('__amd_rocclr')
            c = agg.setdefault(nm, [0, 0.0])
            c[0] += 1
            c[1] += d
    launches = sum(c[0] for c in agg.values())
    print(f'{n} steady iterations (cut at {a.marker}): {launches / n:.1f} launches, '
          f'{copies / n:.2f} device copies (__amd_rocclr_*), {busy / n:.1f} us busy, '
          f'{span / n:.1f} us first-to-last launch per iteration')
    print(f'{"launches/it":>12} {"us/it":>8} {"us/launch":>9}  kernel')
    for nm, (c, d) in agg.items():
        print(f'{c / n:12.2f} {d / n:8.2f} {d / max(c, 1):9.2f}  {nm}')


if __name__ == '__main__':
    main()
