#!/bin/bash
# Round 6, GPU session 23: the update's fused slice reduce with the parameter / moment loads issued
# ahead of the slices; one-round slice sums (BT_REDUCE_ROUNDS=1: twice the blocks) against two.
set -u
cd "$(dirname "$0")/../.."
O=gpurun_out/r6b23
mkdir -p $O
export TMPDIR=/tmp
trap 'find gpurun_out -type f -size +4M -print -delete; du -sh gpurun_out' EXIT
timeout -k 10 300 python -u -m pytest -q --timeout 150 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_adam.py > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; grep -E "^(FAILED|ERROR)" $O/pytest.log | head -20
[ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for e in 2 1; do
    BT_REDUCE_ROUNDS=$e timeout -k 10 200 python bench.py --consumer disc --steps 2000 > $O/disc.log 2>&1 || { tail -5 $O/disc.log; exit 1; }
    grep '^{' $O/disc.log | tee -a $O/disc_rounds$e.jsonl | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'rounds':$e,'disc':d['value'],'ms':d['ms_per_step']}))"
  done
done
bash scripts/gpurun/disc_trace.sh r6b23 > /dev/null || exit 1
BT_REDUCE_ROUNDS=1 bash scripts/gpurun/disc_trace.sh r6b23r1 > /dev/null || exit 1
cp gpurun_out/trace_r6b23/step_sequence.txt $O/disc_step_sequence.txt
cp gpurun_out/trace_r6b23r1/step_sequence.txt $O/disc_step_sequence_rounds1.txt
for f in $O/disc_step_sequence.txt $O/disc_step_sequence_rounds1.txt; do head -1 $f; grep -E "^ +1[345] " $f; done
