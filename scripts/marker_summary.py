#!/usr/bin/env python
"""Summarise rocprofv3 --marker-trace ranges (roctx, BLENDTORCH_ROCTX=1):
count, mean and p90 duration per range name and thread, over the last
``--frac`` of the trace (steady state).

    python scripts/marker_summary.py <dir with *marker_api_trace.csv> [--frac 0.5]"""
import argparse
import csv
import glob
import os
import statistics
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('dir')
    ap.add_argument('--frac', type=float, default=0.5)
    a = ap.parse_args()
    rows = []
    for f in glob.glob(os.path.join(a.dir, '**', '*marker_api_trace.csv'), recursive=True):
        rows += list(csv.DictReader(open(f)))
    if not rows:
        raise SystemExit('no marker_api_trace.csv under ' + a.dir)
    name_key = 'Function' if 'Function' in rows[0] else [k for k in rows[0] if 'name' in k.lower()][0]
    for r in rows:
        r['s'], r['e'] = int(r['Start_Timestamp']), int(r['End_Timestamp'])
    t0 = min(r['s'] for r in rows)
    t1 = max(r['e'] for r in rows)
    lo = t1 - (t1 - t0) * a.frac
    groups = defaultdict(list)
    for r in rows:
        if r['s'] >= lo:
            groups[(r[name_key], r.get('Thread_Id', '?'))].append((r['e'] - r['s']) / 1e3)
    print(f'columns: {list(rows[0].keys())}')
    for (name, tid), d in sorted(groups.items(), key=lambda kv: -sum(kv[1])):
        d.sort()
        print(f'{name:32s} thread {tid:>8}: n={len(d):6d} mean {statistics.mean(d):9.1f} us  '
              f'p90 {d[int(0.9 * (len(d) - 1))]:9.1f} us  total {sum(d) / 1e3:8.1f} ms')


if __name__ == '__main__':
    main()
