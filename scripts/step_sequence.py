#!/usr/bin/env python
"""One steady-state training step from a rocprofv3 kernel trace, kernel by
kernel in launch order: start offset, duration, gap to the previous kernel
and grid size -- so each BN / conv / head kernel can be tied to its layer.
Also the per-kernel mean over the last ``--steps`` steps.

    python scripts/step_sequence.py <dir with *kernel_trace.csv> [--marker adam_update] [--steps 200]

A step is the span between two consecutive launches of ``--marker`` (the
optimizer's update kernel ends every step)."""
import argparse
import csv
import glob
import os
import statistics
from collections import defaultdict


def short(name):
    n = name.replace('(anonymous namespace)::', '').replace('btn::gpu::', '')
    n = n.split('(')[0].replace('void ', '')
    return n[:70]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('dir')
    ap.add_argument('--marker', default='adam_update')
    ap.add_argument('--steps', type=int, default=200)
    a = ap.parse_args()
    rows = []
    for f in glob.glob(os.path.join(a.dir, '**', '*kernel_trace.csv'), recursive=True):
        rows += list(csv.DictReader(open(f)))
    for r in rows:
        r['s'], r['e'] = int(r['Start_Timestamp']), int(r['End_Timestamp'])
        r['k'] = short(r['Kernel_Name'])
    rows.sort(key=lambda r: r['s'])
    ends = [i for i, r in enumerate(rows) if a.marker in r['k']]
    if len(ends) < 3:
        raise SystemExit(f'fewer than 3 {a.marker!r} kernels in the trace')
    steps, lead = [], []
    for i0, i1 in zip(ends[:-1], ends[1:]):
        steps.append(rows[i0 + 1:i1 + 1])
        lead.append(rows[i0 + 1]['s'] - rows[i0]['e'])   # idle GPU time before the step's first kernel
    steps, lead = steps[-a.steps:], lead[-a.steps:]
    # the median-length step, printed in order
    spans = [s[-1]['e'] - s[0]['s'] for s in steps]
    med = sorted(range(len(steps)), key=lambda i: spans[i])[len(steps) // 2]
    st = steps[med]
    t0 = st[0]['s']
    print(f'{len(steps)} steps; median step span {spans[med] / 1e3:.1f} us, mean {statistics.mean(spans) / 1e3:.1f} us; '
          f'kernels per step {len(st)}')
    print(f'{"start":>8} {"dur":>7} {"gap":>6} {"grid":>8}  kernel')
    prev = None
    for r in st:
        gap = (r['s'] - prev) / 1e3 if prev is not None else 0.0
        print(f'{(r["s"] - t0) / 1e3:8.1f} {(r["e"] - r["s"]) / 1e3:7.2f} {gap:6.2f} {r.get("Grid_Size", "?"):>8}  {r["k"]}')
        prev = r['e']
    busy = sum(r['e'] - r['s'] for r in st) / 1e3
    print(f'busy {busy:.1f} us of {spans[med] / 1e3:.1f} us')
    period = [e1[-1]['e'] - e0[-1]['e'] for e0, e1 in zip(steps[:-1], steps[1:])]
    print(f'between steps: median {statistics.median(lead) / 1e3:.1f} us idle before a step\'s first kernel; '
          f'median step period {statistics.median(period) / 1e3:.1f} us')
    # mean per (position in step) over all steps with the same kernel count
    n = len(st)
    same = [s for s in steps if len(s) == n]
    print(f'\nmean over {len(same)} steps with {n} kernels (per position):')
    for j in range(n):
        d = [(s[j]['e'] - s[j]['s']) / 1e3 for s in same]
        print(f'{j:3d} {statistics.mean(d):7.2f} us  {same[0][j]["k"]}')
    tot = defaultdict(float)
    cnt = defaultdict(int)
    for s in steps:
        for r in s:
            tot[r['k']] += (r['e'] - r['s']) / 1e3
            cnt[r['k']] += 1
    print('\nper kernel, summed per step:')
    for k, v in sorted(tot.items(), key=lambda kv: -kv[1]):
        print(f'{v / len(steps):8.2f} us/step {cnt[k] / len(steps):5.2f}x  {k}')


if __name__ == '__main__':
    main()
