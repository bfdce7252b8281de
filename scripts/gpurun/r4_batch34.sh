#!/bin/bash
# GPU session 34: knob sweep on the final defaults -- weight-gradient block target,
# 64-pixel tile threshold.
set -u
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out/b34
export TMPDIR=/tmp
trap 'find gpurun_out -type f -size +4M -print -delete; du -sh gpurun_out' EXIT
for v in "X=0" "BT_WGRAD_BLOCKS=768" "BT_WGRAD_BLOCKS=1024" "BT_WGRAD_BLOCKS=384" "BT_CONV_BM64_BELOW=384" \
         "X=0" "BT_WGRAD_BLOCKS=768" "BT_WGRAD_BLOCKS=1024" "BT_WGRAD_BLOCKS=384" "BT_CONV_BM64_BELOW=384"; do
  timeout -k 10 200 env $v python bench.py --consumer disc --steps 2000 > gpurun_out/b34/sweep.log 2>&1 || { tail -5 gpurun_out/b34/sweep.log; exit 1; }
  grep '^{' gpurun_out/b34/sweep.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'v':'$v','value':d['value'],'ms':d['ms_per_step']}))" | tee -a gpurun_out/b34/sweep.jsonl
done
