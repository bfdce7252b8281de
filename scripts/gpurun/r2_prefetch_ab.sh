#!/bin/bash
# headline bench vs loader depth: posted output buffers (--prefetch) and queued decode launches (--launch-depth),
# on long and driver-style short timed windows
set -u
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
export TMPDIR=/tmp
for cfg in ${CFGS:-"4 2 20 5" "6 2 20 5" "8 2 20 5" "4 2 2000 50" "6 2 2000 50" "8 2 2000 50" "4 2 20 5" "6 2 20 5" "8 2 20 5"}; do
  set -- $cfg
  timeout -k 10 200 python bench.py --steps $3 --warmup $4 --prefetch $1 --launch-depth $2 > gpurun_out/pf.log 2>&1 || { tail -5 gpurun_out/pf.log; exit 1; }
  grep '^{' gpurun_out/pf.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('prefetch=$1 depth=$2 steps=$3', d['value'], d['h2d_gbytes_per_s'], d['gpu_us_per_image'], d['consumer_wait_ms_per_batch'], d['loader_stats']['launches'])"
done
