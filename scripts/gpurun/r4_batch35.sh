#!/bin/bash
# GPU session 35: multi-rank rehearsal on one GPU with the final defaults (gloo,
# 2 ranks sharing the card and its PCIe link): shard and scatter modes.
set -u
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out/b35
export TMPDIR=/tmp
trap 'find gpurun_out -type f -size +4M -print -delete; du -sh gpurun_out' EXIT
for v in "--dist shard" "--dist scatter" "--dist pool"; do
  timeout -k 10 300 python bench.py --gpus 2 --backend gloo --steps 1000 $v > gpurun_out/b35/r2.log 2>&1 || { tail -8 gpurun_out/b35/r2.log; exit 1; }
  grep '^{' gpurun_out/b35/r2.log | tee -a gpurun_out/b35/ranks2.jsonl | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'v':'$v','value':d['value'],'n':d['n_gpus'],'seen':d.get('world_size_seen'),'cpu':d.get('cpu',{}).get('us_per_frame'),'prod':[r.get('producers') for r in d.get('per_rank',[])]}))"
done
