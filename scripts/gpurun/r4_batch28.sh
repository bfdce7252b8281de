#!/bin/bash
# GPU session 28: the disc consumer's busy runtime thread -- HIP graph launch knobs,
# per-thread CPU and throughput each.
set -u
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out/b28
export TMPDIR=/tmp
trap 'find gpurun_out -type f -size +4M -print -delete; du -sh gpurun_out' EXIT
for v in "X=0" "DEBUG_CLR_GRAPH_PACKET_CAPTURE=0" "DEBUG_HIP_GRAPH_BATCH_SIZE=1" "DEBUG_HIP_GRAPH_BATCH_SIZE=64" "X=0"; do
  timeout -k 10 240 env BT_THREAD_REPORT=1 $v python bench.py --consumer disc --steps 2000 > gpurun_out/b28/disc.log 2>&1 || { tail -5 gpurun_out/b28/disc.log; exit 1; }
  grep '^{' gpurun_out/b28/disc.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); c=d.get('cpu',{}); print(json.dumps({'v':'$v','value':d['value'],'ms':d['ms_per_step'],'per':c.get('us_per_frame'),'thr':c.get('threads_cpu_s')[:4]}))" | tee -a gpurun_out/b28/disc.jsonl
done
