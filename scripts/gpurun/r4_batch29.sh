#!/bin/bash
# GPU session 29: is the disc consumer's busy runtime thread the copy engines'
# completion handling?  Direct reads instead of DMA copies; blit-kernel copies.
set -u
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out/b29
export TMPDIR=/tmp
trap 'find gpurun_out -type f -size +4M -print -delete; du -sh gpurun_out' EXIT
for v in "X=0 --h2d copy" "X=0 --h2d auto" "HSA_ENABLE_SDMA=0 --h2d copy"; do
  e=${v%% *}; a=${v#* }
  timeout -k 10 240 env BT_THREAD_REPORT=1 $e python bench.py --consumer disc --steps 2000 $a > gpurun_out/b29/disc.log 2>&1 || { tail -5 gpurun_out/b29/disc.log; exit 1; }
  grep '^{' gpurun_out/b29/disc.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); c=d.get('cpu',{}); print(json.dumps({'v':'$v','value':d['value'],'ms':d['ms_per_step'],'per':c.get('us_per_frame'),'thr':c.get('threads_cpu_s')[:4]}))" | tee -a gpurun_out/b29/disc.jsonl
done
