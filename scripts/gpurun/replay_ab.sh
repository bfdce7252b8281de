#!/bin/bash
# Replay sampler: value-transform policy A/B (table / arithmetic / auto), batch 8 and 64, + kernel stats
set -u
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
export TMPDIR=/tmp
for x in 0 1 auto; do
  for args in "--batch 8" "--batch 64 --steps 500"; do
    BLENDTORCH_DECODE_XFORM=$x timeout -k 10 120 python benchmarks/bench_replay.py $args > gpurun_out/replay_ab.log 2>&1 || { tail -5 gpurun_out/replay_ab.log; exit 1; }
    grep '^{' gpurun_out/replay_ab.log | python -c "
import json,sys
d=json.loads(sys.stdin.read()); print('xform=$x', 'B', d['batch'], d['us_per_batch'], 'us', d['effective_tbps'], 'TB/s')"
  done
done
for x in 0 auto; do
  BLENDTORCH_DECODE_XFORM=$x timeout -k 10 120 rocprofv3 --kernel-trace --stats -d /tmp/rp_rab_$x -o run --output-format csv -- python benchmarks/bench_replay.py --batch 64 --steps 300 > gpurun_out/rab_$x.log 2>&1 || exit 1
  f=$(find /tmp/rp_rab_$x -name '*kernel_stats.csv' | head -1)
  echo "xform=$x"; head -3 "$f" | cut -c1-200
done
