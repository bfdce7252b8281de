#!/bin/bash
# GPU session 36: disc consumer loader depth (posted buffers = graphs per ring tensor - 2).
set -u
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out/b36
export TMPDIR=/tmp
trap 'find gpurun_out -type f -size +4M -print -delete; du -sh gpurun_out' EXIT
for v in "" "--prefetch 8" "--prefetch 4" "--copy-streams 2" "" "--prefetch 8" "--prefetch 4" "--copy-streams 2"; do
  timeout -k 10 200 python bench.py --consumer disc --steps 2000 $v > gpurun_out/b36/sweep.log 2>&1 || { tail -5 gpurun_out/b36/sweep.log; exit 1; }
  grep '^{' gpurun_out/b36/sweep.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'v':'$v','value':d['value'],'ms':d['ms_per_step']}))" | tee -a gpurun_out/b36/sweep.jsonl
done
