#!/bin/bash
# GPU session 20: where the consumer process's CPU per frame goes (loader worker
# stages with BT_LOADER_CPU=1, per-thread CPU), and the headline without accounting.
set -u
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out/b20
export TMPDIR=/tmp
trap 'find gpurun_out -type f -size +4M -print -delete; du -sh gpurun_out' EXIT
for v in "BT_LOADER_CPU=1" "X=0" "BT_LOADER_CPU=1 BT_LOADER_POLL_US=100"; do
  timeout -k 10 240 env BT_THREAD_REPORT=1 $v python bench.py --steps 2000 > gpurun_out/b20/headline.log 2>&1 || { tail -5 gpurun_out/b20/headline.log; exit 1; }
  grep '^{' gpurun_out/b20/headline.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'v':'$v','value':d['value'],'cpu':d.get('cpu')}))" | tee -a gpurun_out/b20/headline.jsonl
done
