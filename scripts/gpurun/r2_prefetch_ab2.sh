#!/bin/bash
# posted loader buffers 6 vs 8, alternating, on driver-style short and long timed windows
set -u
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
export TMPDIR=/tmp
while read -r pf steps warm; do
  timeout -k 10 200 python bench.py --steps $steps --warmup $warm --prefetch $pf > gpurun_out/pf.log 2>&1 || { tail -5 gpurun_out/pf.log; exit 1; }
  grep '^{' gpurun_out/pf.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('prefetch=$pf steps=$steps', d['value'], d['h2d_gbytes_per_s'], d['gpu_us_per_image'], d['loader_stats']['launches'])"
done <<'LIST'
6 20 5
8 20 5
6 2000 50
8 2000 50
6 20 5
8 20 5
6 2000 50
8 2000 50
6 20 5
8 20 5
LIST
