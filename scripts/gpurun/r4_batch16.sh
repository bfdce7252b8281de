#!/bin/bash
# GPU session 16: 64-pixel tiles for more of the tap GEMMs (BT_CONV_BM64_BELOW) -- A/B and traces.
set -u
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out/b16
export TMPDIR=/tmp
trap 'find gpurun_out -type f -size +4M -print -delete; du -sh gpurun_out' EXIT
for v in "X=0" "BT_CONV_BM64_BELOW=768" "BT_CONV_BM64_BELOW=1300" "X=1" "BT_CONV_BM64_BELOW=768" "BT_CONV_BM64_BELOW=1300"; do
  timeout -k 10 200 env $v python bench.py --consumer disc --steps 2000 > gpurun_out/b16/sweep.log 2>&1 || { tail -5 gpurun_out/b16/sweep.log; exit 1; }
  grep '^{' gpurun_out/b16/sweep.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'v':'$v','value':d['value'],'ms':d['ms_per_step']}))" | tee -a gpurun_out/b16/sweep.jsonl
done
for v in 768 1300; do
  BT_CONV_BM64_BELOW=$v bash scripts/gpurun/disc_trace.sh r4p_$v > /dev/null || exit 1
  cp gpurun_out/trace_r4p_$v/step_sequence.txt gpurun_out/b16/step_sequence_$v.txt
  echo "== $v"; sed -n '/mean over/,/per kernel/p' gpurun_out/trace_r4p_$v/step_sequence.txt | head -26
done
