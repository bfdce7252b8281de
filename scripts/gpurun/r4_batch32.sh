#!/bin/bash
# GPU session 32: BN apply grid cap (folding applies: 1024 blocks left BN2 at 1.17
# passes per block) -- BN tests, disc A/B, trace of the best.
set -u
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out/b32
export TMPDIR=/tmp
trap 'find gpurun_out -type f -size +4M -print -delete; du -sh gpurun_out' EXIT
for v in "X=0" "BT_BN_FOLD_GRID=512" "BT_BN_FOLD_GRID=768" "X=0" "BT_BN_FOLD_GRID=512" "BT_BN_FOLD_GRID=768"; do
  timeout -k 10 200 env $v python bench.py --consumer disc --steps 2000 > gpurun_out/b32/sweep.log 2>&1 || { tail -5 gpurun_out/b32/sweep.log; exit 1; }
  grep '^{' gpurun_out/b32/sweep.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'v':'$v','value':d['value'],'ms':d['ms_per_step']}))" | tee -a gpurun_out/b32/sweep.jsonl
done
BT_BN_FOLD_GRID=512 bash scripts/gpurun/disc_trace.sh r4t > /dev/null || exit 1
cp gpurun_out/trace_r4t/step_sequence.txt gpurun_out/b32/
sed -n '/mean over/,/per kernel/p' gpurun_out/trace_r4t/step_sequence.txt | head -26
