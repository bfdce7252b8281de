#!/bin/bash
# Round 6, GPU session 20: the backward's last slice reduce summed inside the Adam update launch
# (FusedAdam.attach_reduce; the schedule then rides in the first fused data + weight gradient
# launch): adam / conv / consumer / densityopt tests, disc A/B alternating, trace.
set -u
cd "$(dirname "$0")/../.."
O=gpurun_out/r6b20
mkdir -p $O
export TMPDIR=/tmp
trap 'find gpurun_out -type f -size +4M -print -delete; du -sh gpurun_out' EXIT
timeout -k 10 600 python -u -m pytest -q --timeout 150 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_adam.py tests/test_gpu_consumer.py tests/test_densityopt.py > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; grep -E "^(FAILED|ERROR)" $O/pytest.log | head -20
[ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do
  for e in 1 0; do
    BT_ADAM_FUSE_REDUCE=$e timeout -k 10 200 python bench.py --consumer disc --steps 2000 > $O/disc.log 2>&1 || { tail -5 $O/disc.log; exit 1; }
    grep '^{' $O/disc.log | tee -a $O/disc_fuse$e.jsonl | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'fuse':$e,'disc':d['value'],'ms':d['ms_per_step']}))"
  done
done
bash scripts/gpurun/disc_trace.sh r6b20 > /dev/null || exit 1
cp gpurun_out/trace_r6b20/step_sequence.txt $O/disc_step_sequence.txt
grep -A19 "mean over" $O/disc_step_sequence.txt | head -20; head -1 $O/disc_step_sequence.txt
