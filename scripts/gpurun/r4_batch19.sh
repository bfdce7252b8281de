#!/bin/bash
# GPU session 19: CPU per delivered frame -- producer render cost on the box CPU,
# headline with named per-thread CPU, loader completion-poll grain A/B.
set -u
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out/b19
export TMPDIR=/tmp
trap 'find gpurun_out -type f -size +4M -print -delete; du -sh gpurun_out' EXIT
(cd pytorch-blender_amd/blendtorch/bin && timeout -k 10 60 ./cubesim --bench 3000 --mode rgba) | tee gpurun_out/b19/cubesim_bench.json
for v in "X=0" "BT_LOADER_POLL_US=50" "BT_LOADER_POLL_US=200" "X=1"; do
  timeout -k 10 240 env BT_THREAD_REPORT=1 $v python bench.py --steps 2000 > gpurun_out/b19/headline.log 2>&1 || { tail -5 gpurun_out/b19/headline.log; exit 1; }
  grep '^{' gpurun_out/b19/headline.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'v':'$v','value':d['value'],'cpu':d.get('cpu')}))" | tee -a gpurun_out/b19/headline.jsonl
done
