#!/bin/bash
# Round 5, GPU session 14 (fence-free grid barrier): the first BN applied by the u8 first layer's own
# kernel after a grid barrier (BT_CONV1_BN), the head's fp64 BN sums
# (deterministic step), and the disc A/B of both against the apply launches.
set -u
cd "$(dirname "$0")/../.."
O=gpurun_out/r5b14
mkdir -p $O
export TMPDIR=/tmp
trap 'find gpurun_out -type f -size +4M -print -delete; du -sh gpurun_out' EXIT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_conv_wgrad.py -k "applies_its or first_layer or deferred" -m gpu > $O/pytest_new.log 2>&1 || { tail -40 $O/pytest_new.log; exit 1; }
tail -2 $O/pytest_new.log
for v in "outbn:" "applybn:BT_CONV1_BN=0 BT_CONV_OUT_BN=0" "conv1only:BT_CONV_OUT_BN=0" "outbn:" "applybn:BT_CONV1_BN=0 BT_CONV_OUT_BN=0" "conv1only:BT_CONV_OUT_BN=0"; do
  name=${v%%:*}; e=${v#*:}
  timeout -k 10 200 env $e python bench.py --consumer disc --steps 2000 > $O/disc.log 2>&1 || { tail -5 $O/disc.log; exit 1; }
  grep '^{' $O/disc.log | tee -a $O/disc_$name.jsonl | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'v':'$name','disc':d['value'],'ms':d['ms_per_step']}))"
done
bash scripts/gpurun/disc_trace.sh r5b14 > /dev/null || exit 1
cp gpurun_out/trace_r5b14/step_sequence.txt $O/disc_step_sequence.txt
grep -A22 "mean over" $O/disc_step_sequence.txt
grep "busy\|median step" $O/disc_step_sequence.txt
