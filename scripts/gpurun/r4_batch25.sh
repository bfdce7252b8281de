#!/bin/bash
# GPU session 25: host-ordered hand-off as the headline default -- short (20-step)
# and long (2000-step) windows, 3 repeats each, against the device-ordered default.
set -u
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out/b25
export TMPDIR=/tmp
trap 'find gpurun_out -type f -size +4M -print -delete; du -sh gpurun_out' EXIT
for rep in 1 2 3; do
for st in 20 2000; do
for v in "--host-sync off --prefetch 6" "--host-sync on --prefetch 12" "--host-sync on --prefetch 8"; do
  timeout -k 10 240 python bench.py --steps $st --warmup 10 $v > gpurun_out/b25/headline.log 2>&1 || { tail -5 gpurun_out/b25/headline.log; exit 1; }
  grep '^{' gpurun_out/b25/headline.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); c=d.get('cpu',{}); print(json.dumps({'v':'$v','steps':$st,'value':d['value'],'per':c.get('us_per_frame')}))" | tee -a gpurun_out/b25/headline.jsonl
done; done; done
