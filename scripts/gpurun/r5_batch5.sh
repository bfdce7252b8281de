#!/bin/bash
# Round 5, GPU session 5: the head's loss wave with its partial loads in
# flight together, the one-launch Adam with the schedule worked out ahead
# (A/B), a step trace, and the first layer's weight gradient alone.
set -u
cd "$(dirname "$0")/../.."
O=gpurun_out/r5b5
mkdir -p $O
export TMPDIR=/tmp
trap 'find gpurun_out -type f -size +4M -print -delete; du -sh gpurun_out' EXIT
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_consumer.py tests/test_adam.py -m gpu > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for v in "base:" "adam1:BT_ADAM_ONE_LAUNCH=1" "base:" "adam1:BT_ADAM_ONE_LAUNCH=1"; do
  name=${v%%:*}; e=${v#*:}
  timeout -k 10 200 env $e python bench.py --consumer disc --steps 2000 > $O/disc.log 2>&1 || { tail -5 $O/disc.log; exit 1; }
  grep '^{' $O/disc.log | tee -a $O/disc_$name.jsonl | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'v':'$name','disc':d['value'],'ms':d['ms_per_step']}))"
done
bash scripts/gpurun/disc_trace.sh r5b5 > /dev/null || exit 1
cp gpurun_out/trace_r5b5/step_sequence.txt $O/disc_step_sequence.txt
grep -A23 "mean over" $O/disc_step_sequence.txt
BT_ADAM_ONE_LAUNCH=1 bash scripts/gpurun/disc_trace.sh r5b5a > /dev/null || exit 1
cp gpurun_out/trace_r5b5a/step_sequence.txt $O/disc_step_sequence_adam1.txt
grep -A23 "mean over" $O/disc_step_sequence_adam1.txt | tail -4
timeout -k 10 600 python scripts/c4w_bench.py --iters 200 > $O/c4w_bench.jsonl 2>&1 || { tail -5 $O/c4w_bench.jsonl; exit 1; }
cat $O/c4w_bench.jsonl
