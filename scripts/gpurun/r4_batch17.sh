#!/bin/bash
# GPU session 17: bigger tap-GEMM tiles -- 128-pixel tiles for every layer, 128-channel tiles for the deep layers.
set -u
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out/b17
export TMPDIR=/tmp
trap 'find gpurun_out -type f -size +4M -print -delete; du -sh gpurun_out' EXIT
for v in "X=0" "BT_CONV_BM64_BELOW=200" "BT_CONV_BN=128" "BT_CONV_BN=128 BT_CONV_BM64_BELOW=200" "X=1" "BT_CONV_BM64_BELOW=200" "BT_CONV_BN=128"; do
  timeout -k 10 200 env $v python bench.py --consumer disc --steps 2000 > gpurun_out/b17/sweep.log 2>&1 || { tail -5 gpurun_out/b17/sweep.log; exit 1; }
  grep '^{' gpurun_out/b17/sweep.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'v':'$v','value':d['value'],'ms':d['ms_per_step']}))" | tee -a gpurun_out/b17/sweep.jsonl
done
for v in "BT_CONV_BM64_BELOW=200" "BT_CONV_BN=128"; do
  tag=r4q_${v/=/_}
  env $v bash scripts/gpurun/disc_trace.sh $tag > /dev/null || exit 1
  cp gpurun_out/trace_$tag/step_sequence.txt gpurun_out/b17/step_sequence_${v/=/_}.txt
  echo "== $v"; sed -n '/mean over/,/per kernel/p' gpurun_out/trace_$tag/step_sequence.txt | head -26
done
