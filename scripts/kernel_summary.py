#!/usr/bin/env python
"""Per-kernel totals from a rocprofv3 kernel trace, normalised per iteration:
launches and device time per iteration for every kernel name, in first-launch
order, plus the busy time per iteration.  For loops whose iteration has no
single marker kernel (densityopt: two optimizer updates per iteration).

    python scripts/kernel_summary.py <dir with *kernel_trace.csv> --iters N [--skip-frac 0.1]
"""
import argparse
import csv
import glob
import os
from collections import OrderedDict


def short(name):
    n = name.replace('(anonymous namespace)::', '').replace('btn::gpu::', '')
    return n.split('(')[0].replace('void ', '')[:80]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('dir')
    ap.add_argument('--iters', type=int, required=True, help='iterations the traced run executed')
    ap.add_argument('--skip-frac', type=float, default=0.1, help='leading fraction of launches dropped (warm-up, capture)')
    a = ap.parse_args()
    rows = []
    for f in glob.glob(os.path.join(a.dir, '**', '*kernel_trace.csv'), recursive=True):
        rows += list(csv.DictReader(open(f)))
    rows.sort(key=lambda r: int(r['Start_Timestamp']))
    skip = int(len(rows) * a.skip_frac)
    kept = rows[skip:]
    iters = a.iters * (1 - a.skip_frac)
    agg = OrderedDict()
    for r in kept:
        k = short(r['Kernel_Name'])
        d = (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) * 1e-3
        c = agg.setdefault(k, [0, 0.0])
        c[0] += 1
        c[1] += d
    span = (int(kept[-1]['End_Timestamp']) - int(kept[0]['Start_Timestamp'])) * 1e-3 if kept else 0.0
    busy = sum(v[1] for v in agg.values())
    print(f'{len(kept)} launches over ~{iters:.0f} iterations: {len(kept) / iters:.1f} kernels, '
          f'{busy / iters:.1f} us busy per iteration, wall span {span / iters:.1f} us per iteration')
    print(f"{'launches/it':>11s} {'us/it':>8s} {'us/launch':>9s}  kernel")
    for k, (n, d) in agg.items():
        print(f'{n / iters:11.2f} {d / iters:8.2f} {d / n:9.2f}  {k}')


if __name__ == '__main__':
    main()
