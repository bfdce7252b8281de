#!/bin/bash
# Round 5, GPU session 12: the last BN's backward applied inside the fused
# head (sums worked out in the head forward, factored through dlogit) against
# the accumulator + apply-launch path, and the step trace.
set -u
cd "$(dirname "$0")/../.."
O=gpurun_out/r5b12
mkdir -p $O
export TMPDIR=/tmp
trap 'find gpurun_out -type f -size +4M -print -delete; du -sh gpurun_out' EXIT
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_consumer.py tests/test_conv_wgrad.py tests/test_adam.py -m gpu > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for v in "headbn:" "applybn:BT_HEAD_BN_BWD=0" "headbn:" "applybn:BT_HEAD_BN_BWD=0"; do
  name=${v%%:*}; e=${v#*:}
  timeout -k 10 200 env $e python bench.py --consumer disc --steps 2000 > $O/disc.log 2>&1 || { tail -5 $O/disc.log; exit 1; }
  grep '^{' $O/disc.log | tee -a $O/disc_$name.jsonl | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'v':'$name','disc':d['value'],'ms':d['ms_per_step']}))"
done
bash scripts/gpurun/disc_trace.sh r5b12 > /dev/null || exit 1
cp gpurun_out/trace_r5b12/step_sequence.txt $O/disc_step_sequence.txt
grep -A20 "mean over" $O/disc_step_sequence.txt
grep "busy\|median step" $O/disc_step_sequence.txt
