#!/bin/bash
# Round 6, GPU session 13: the data-gradient epilogue's BN inputs and the head backward's per-channel
# inputs / dlogit as loads issued together (no round trips in series): GPU suite, disc x3 + trace,
# headline bench x2.
set -u
cd "$(dirname "$0")/../.."
O=gpurun_out/r6b13
mkdir -p $O
export TMPDIR=/tmp
trap 'find gpurun_out -type f -size +4M -print -delete; du -sh gpurun_out' EXIT
timeout -k 10 700 python -u -m pytest -q --timeout 150 --timeout-method thread -p no:cacheprovider -m gpu tests \
  > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; grep -E "^(FAILED|ERROR)" $O/pytest.log | head -20
[ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do
  timeout -k 10 200 python bench.py --consumer disc --steps 2000 > $O/disc.log 2>&1 || { tail -5 $O/disc.log; exit 1; }
  grep '^{' $O/disc.log | tee -a $O/disc_default.jsonl | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'disc':d['value'],'ms':d['ms_per_step']}))"
done
bash scripts/gpurun/disc_trace.sh r6b13 > /dev/null || exit 1
cp gpurun_out/trace_r6b13/step_sequence.txt $O/disc_step_sequence.txt
grep -A19 "mean over" $O/disc_step_sequence.txt | head -20
for i in 1 2; do
  timeout -k 10 300 python bench.py > $O/bench_default.log 2>&1 || { tail -5 $O/bench_default.log; exit 1; }
  grep '^{' $O/bench_default.log | tee -a $O/bench_default.jsonl | cut -c1-150
done
