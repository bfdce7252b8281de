#!/usr/bin/env python
"""Summarise a rocprofv3 kernel (+ memory-copy) trace as per-queue busy time
and the idle gaps of the busiest queue over the steady-state window.

    python scripts/trace_timeline.py <dir with *kernel_trace.csv> [--skip-frac 0.3]

Prints, per queue: kernels, busy us, share of the window; the top kernels by
time on the busiest queue; the distribution of idle gaps between its kernels
(what the consumer stream waits for); and DMA copy totals if traced."""
import argparse
import csv
import glob
import os
import statistics
from collections import defaultdict


def load(pattern):
    rows = []
    for f in glob.glob(pattern, recursive=True):
        with open(f) as fp:
            rows += list(csv.DictReader(fp))
    return rows


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('dir')
    ap.add_argument('--skip-frac', type=float, default=0.3, help='leading fraction of the trace skipped (warm-up)')
    ap.add_argument('--last', type=int, default=0, help='analyse only the last N kernels (steady state)')
    a = ap.parse_args()
    ks = load(os.path.join(a.dir, '**', '*kernel_trace.csv'))
    if not ks:
        raise SystemExit('no kernel_trace.csv under ' + a.dir)
    for r in ks:
        r['s'], r['e'] = int(r['Start_Timestamp']), int(r['End_Timestamp'])
    ks.sort(key=lambda r: r['s'])
    if a.last:
        ks = ks[-a.last:]
        lo = ks[0]['s']
    else:
        t0, t1 = ks[0]['s'], ks[-1]['e']
        lo = t0 + int((t1 - t0) * a.skip_frac)
        ks = [r for r in ks if r['s'] >= lo]
    span = (ks[-1]['e'] - ks[0]['s']) / 1e3
    byq = defaultdict(list)
    for r in ks:
        byq[r.get('Queue_Id', '?')].append(r)
    print(f'window {span:.0f} us, {len(ks)} kernels')
    for q, rs in sorted(byq.items(), key=lambda kv: -sum(r["e"] - r["s"] for r in kv[1])):
        busy = sum(r['e'] - r['s'] for r in rs) / 1e3
        print(f'queue {q}: {len(rs)} kernels, busy {busy:.0f} us ({100 * busy / span:.1f}%)')
    q = max(byq, key=lambda k: sum(r['e'] - r['s'] for r in byq[k]))
    rs = byq[q]
    tot = defaultdict(lambda: [0, 0])
    for r in rs:
        n = r['Kernel_Name'][:90]
        tot[n][0] += 1
        tot[n][1] += r['e'] - r['s']
    print(f'\ntop kernels on queue {q}:')
    for n, (c, t) in sorted(tot.items(), key=lambda kv: -kv[1][1])[:25]:
        print(f'  {t / 1e3:9.0f} us  {c:6d}x  {t / 1e3 / c:8.2f} us/call  {n}')
    gaps = [(b['s'] - x['e']) / 1e3 for x, b in zip(rs, rs[1:]) if b['s'] > x['e']]
    if gaps:
        gaps.sort()
        big = [g for g in gaps if g > 20]
        print(f'\nidle gaps on queue {q}: n={len(gaps)} total {sum(gaps):.0f} us, median {statistics.median(gaps):.1f} us, '
              f'p99 {gaps[int(0.99 * (len(gaps) - 1))]:.1f} us; gaps > 20 us: {len(big)} totalling {sum(big):.0f} us')
    for qq, rr in byq.items():
        if qq != q:
            names = defaultdict(lambda: [0, 0])
            for r in rr:
                names[r['Kernel_Name'][:70]][0] += 1
                names[r['Kernel_Name'][:70]][1] += r['e'] - r['s']
            print(f'\nqueue {qq}: ' + '; '.join(f'{n} {c}x {t / 1e3 / c:.1f} us' for n, (c, t) in names.items()))
    cs = load(os.path.join(a.dir, '**', '*memory_copy_trace.csv'))
    if cs:
        if cs and 'Size' not in cs[0]:
            print('memory copy columns:', list(cs[0].keys()))
        cs = [c for c in cs if int(c['Start_Timestamp']) >= lo]
        nbytes = sum(int(c.get('Size', 0) or 0) for c in cs)
        busy = sum(int(c['End_Timestamp']) - int(c['Start_Timestamp']) for c in cs) / 1e3
        print(f'\nmemory copies in window: {len(cs)}, {nbytes / 1e6:.0f} MB, summed copy time {busy:.0f} us '
              f'({nbytes / 1e3 / max(busy, 1e-9):.1f} GB/s per copy)')


if __name__ == '__main__':
    main()
