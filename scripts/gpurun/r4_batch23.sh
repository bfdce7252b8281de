#!/bin/bash
# GPU session 23: headline with host-ordered loader hand-off (no cross-stream
# event waits) vs device-ordered, per-thread CPU each.
set -u
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out/b23
export TMPDIR=/tmp
trap 'find gpurun_out -type f -size +4M -print -delete; du -sh gpurun_out' EXIT
for v in "--host-sync off" "--host-sync on" "--host-sync on --prefetch 8" "--host-sync off"; do
  timeout -k 10 240 env BT_THREAD_REPORT=1 BT_LOADER_CPU=1 python bench.py --steps 2000 $v > gpurun_out/b23/headline.log 2>&1 || { tail -5 gpurun_out/b23/headline.log; exit 1; }
  grep '^{' gpurun_out/b23/headline.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); c=d.get('cpu',{}); print(json.dumps({'v':'$v','value':d['value'],'per':c.get('us_per_frame'),'loader':c.get('loader_us_per_frame'),'thr':c.get('threads_cpu_s')}))" | tee -a gpurun_out/b23/headline.jsonl
done
