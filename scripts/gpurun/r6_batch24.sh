#!/bin/bash
# Round 6, GPU session 24: the update's fused slice sum at 4 loads per round (58 VGPRs: 8 waves per
# SIMD for the whole update launch, two round trips) against 8 (92 VGPRs, one round trip).
set -u
cd "$(dirname "$0")/../.."
O=gpurun_out/r6b24
mkdir -p $O
export TMPDIR=/tmp
trap 'find gpurun_out -type f -size +4M -print -delete; du -sh gpurun_out' EXIT
BT_ADAM_FR_SG=4 timeout -k 10 300 python -u -m pytest -q --timeout 150 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_adam.py -k "reduce" > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; grep -E "^(FAILED|ERROR)" $O/pytest.log | head -20
[ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do
  for e in 4 8; do
    BT_ADAM_FR_SG=$e timeout -k 10 200 python bench.py --consumer disc --steps 2000 > $O/disc.log 2>&1 || { tail -5 $O/disc.log; exit 1; }
    grep '^{' $O/disc.log | tee -a $O/disc_sg$e.jsonl | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'sg':$e,'disc':d['value'],'ms':d['ms_per_step']}))"
  done
done
BT_ADAM_FR_SG=4 bash scripts/gpurun/disc_trace.sh r6b24s4 > /dev/null || exit 1
BT_ADAM_FR_SG=8 bash scripts/gpurun/disc_trace.sh r6b24s8 > /dev/null || exit 1
cp gpurun_out/trace_r6b24s4/step_sequence.txt $O/disc_step_sequence_sg4.txt
cp gpurun_out/trace_r6b24s8/step_sequence.txt $O/disc_step_sequence_sg8.txt
for f in $O/disc_step_sequence_sg4.txt $O/disc_step_sequence_sg8.txt; do head -1 $f; grep -E "^ +1[45] " $f; done
