#!/bin/bash
# GPU session 21: which runtime thread spins a core under the headline stream --
# completion-query throttle and ROCclr / ROCr wait knobs, per-thread CPU each.
set -u
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out/b21
export TMPDIR=/tmp
trap 'find gpurun_out -type f -size +4M -print -delete; du -sh gpurun_out' EXIT
for v in "X=0" "BT_LOADER_REAP_US=500" "ROC_ACTIVE_WAIT_TIMEOUT=0" "HSA_ENABLE_MWAITX=1" "BT_LOADER_REAP_US=2000"; do
  timeout -k 10 240 env BT_THREAD_REPORT=1 BT_LOADER_CPU=1 $v python bench.py --steps 2000 > gpurun_out/b21/headline.log 2>&1 || { tail -5 gpurun_out/b21/headline.log; exit 1; }
  grep '^{' gpurun_out/b21/headline.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); c=d.get('cpu',{}); print(json.dumps({'v':'$v','value':d['value'],'per':c.get('us_per_frame'),'loader':c.get('loader_us_per_frame'),'thr':c.get('threads_cpu_s')}))" | tee -a gpurun_out/b21/headline.jsonl
done
