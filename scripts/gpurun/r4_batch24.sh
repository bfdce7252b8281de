#!/bin/bash
# GPU session 24: host-ordered hand-off -- recover the throughput (prefetch,
# launch depth, poll grain) at its CPU per frame.
set -u
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out/b24
export TMPDIR=/tmp
trap 'find gpurun_out -type f -size +4M -print -delete; du -sh gpurun_out' EXIT
for v in "X=0 --host-sync off" "X=0 --host-sync on --prefetch 8" "X=0 --host-sync on --prefetch 8 --launch-depth 3" \
         "X=0 --host-sync on --prefetch 12" "BT_LOADER_POLL_US=4 --host-sync on --prefetch 8" \
         "X=0 --host-sync on --prefetch 16 --launch-depth 3" "X=0 --host-sync off"; do
  e=${v%% *}; a=${v#* }
  timeout -k 10 240 env BT_THREAD_REPORT=1 $e python bench.py --steps 2000 $a > gpurun_out/b24/headline.log 2>&1 || { tail -5 gpurun_out/b24/headline.log; exit 1; }
  grep '^{' gpurun_out/b24/headline.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); c=d.get('cpu',{}); print(json.dumps({'v':'$v','value':d['value'],'per':c.get('us_per_frame'),'thr':c.get('threads_cpu_s')}))" | tee -a gpurun_out/b24/headline.jsonl
done
