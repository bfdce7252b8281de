#!/bin/bash
# GPU session 26: the new headline defaults (host-ordered hand-off, 8 posted
# buffers, producers from the r4 per-frame CPU costs) vs 7 / 8 producers; disc check.
set -u
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out/b26
export TMPDIR=/tmp
trap 'find gpurun_out -type f -size +4M -print -delete; du -sh gpurun_out' EXIT
for v in "" "--producers 7" "--producers 8" "" "--producers 7" "--producers 8"; do
  timeout -k 10 240 env BT_THREAD_REPORT=1 python bench.py --steps 2000 $v > gpurun_out/b26/headline.log 2>&1 || { tail -5 gpurun_out/b26/headline.log; exit 1; }
  grep '^{' gpurun_out/b26/headline.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); c=d.get('cpu',{}); print(json.dumps({'v':'$v','value':d['value'],'producers':[r.get('producers') for r in d.get('per_rank', [])],'per':c.get('us_per_frame'),'thr':c.get('threads_cpu_s')}))" | tee -a gpurun_out/b26/headline.jsonl
done
timeout -k 10 240 python bench.py --consumer disc --steps 2000 > gpurun_out/b26/disc.log 2>&1 || { tail -5 gpurun_out/b26/disc.log; exit 1; }
grep '^{' gpurun_out/b26/disc.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); c=d.get('cpu',{}); print(json.dumps({'v':'disc','value':d['value'],'ms':d['ms_per_step'],'per':c.get('us_per_frame')}))" | tee -a gpurun_out/b26/headline.jsonl
