#!/bin/bash
# headline bench vs loader depth: posted output buffers (--prefetch) and queued decode launches (--launch-depth)
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
for cfg in ${CFGS:-"16 2" "16 3" "24 4" "16 2" "16 3" "24 4"}; do
  set -- $cfg
  timeout -k 10 200 python bench.py --steps 4000 --prefetch $1 --launch-depth $2 > gpurun_out/pf.log 2>&1 || { tail -5 gpurun_out/pf.log; exit 1; }
  grep '^{' gpurun_out/pf.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('prefetch=$1 depth=$2', d['value'], d['h2d_gbytes_per_s'], d['gpu_us_per_image'], d['consumer_wait_ms_per_batch'], d['loader_stats']['launches'])"
done
