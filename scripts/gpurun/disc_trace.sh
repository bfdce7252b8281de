#!/bin/bash
# Kernel trace of bench.py --consumer disc (1 GPU, no process group): per-step kernel times
set -u
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/dtr -o run -- python3 bench.py --consumer disc --steps 600 ${BENCH_ARGS:-} > gpurun_out/dtr.log 2>&1 || { tail gpurun_out/dtr.log; exit 1; }
grep '^{' gpurun_out/dtr.log | cut -c1-200
f=$(find /tmp/dtr -name '*kernel_trace.csv' | head -1)
python3 - "$f" <<'PY' | tee gpurun_out/disc_trace_summary.txt
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r['Start_Timestamp']))
# steady state: the last 300 optimizer steps on the step's queue
ad = [i for i, r in enumerate(rows) if 'adam_update' in r['Kernel_Name']]
lo, hi = ad[-301], ad[-1]
win = rows[lo + 1:hi + 1]
steps = 300
tot = collections.defaultdict(float); cnt = collections.Counter()
for r in win:
    n = r['Kernel_Name'].replace('(anonymous namespace)::', '').split('(')[0].replace('void ', '')[:80]
    tot[n] += (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1000
    cnt[n] += 1
span = (int(win[-1]['End_Timestamp']) - int(win[0]['Start_Timestamp'])) / 1000
busy = sum(tot.values())
print(f'{steps} steps: {span / steps:.1f} us/step span, kernels busy {busy / steps:.1f} us/step, {len(win) / steps:.1f} kernels/step')
for k, v in sorted(tot.items(), key=lambda kv: -kv[1]):
    print(f'{v / steps:8.2f} us/step {cnt[k] / steps:5.2f}x {v / cnt[k]:8.2f} us/call  {k}')
PY
