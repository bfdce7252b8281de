#!/bin/bash
# GPU session 8: where the BN applies run -- bench A/B of the placements in one box, traces, PMC of the default.
set -u
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
export TMPDIR=/tmp
trap 'find gpurun_out -type f -size +4M -print -delete; du -sh gpurun_out' EXIT
for v in "X=0" "BT_LAZY_HEAD_BN=0" "BT_LAZY_CONV_BN=1" "BT_DEFER_BN_BWD=1" "BT_LAZY_CONV_BN=1 BT_DEFER_BN_BWD=1" "X=0"; do
  timeout -k 10 200 env $v python bench.py --consumer disc --steps 2000 > gpurun_out/sweep8.log 2>&1 || { tail -5 gpurun_out/sweep8.log; exit 1; }
  grep '^{' gpurun_out/sweep8.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'v':'$v','value':d['value'],'ms':d['ms_per_step']}))" | tee -a gpurun_out/sweep8.jsonl
done
bash scripts/gpurun/disc_trace.sh r4i > /dev/null || exit 1
sed -n '/mean over/,$p' gpurun_out/trace_r4i/step_sequence.txt | head -40
BT_LAZY_HEAD_BN=0 bash scripts/gpurun/disc_trace.sh r4i_nolazy > /dev/null || exit 1
sed -n '/mean over/,$p' gpurun_out/trace_r4i_nolazy/step_sequence.txt | head -30
bash scripts/gpurun/disc_pmc.sh > /dev/null || exit 1
cat gpurun_out/disc_pmc/summary.txt
