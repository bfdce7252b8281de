#!/bin/bash
# Round 6, GPU session 11: memory-counter waits that count exactly (unconditional buffer loads / stores,
# loads issued in consumption order) in the first layer's forward and weight gradient, every class's weights
# loaded up front in the patch data gradient: tests, c4p bench, disc x3, trace.
set -u
cd "$(dirname "$0")/../.."
O=gpurun_out/r6b11
mkdir -p $O
export TMPDIR=/tmp
trap 'find gpurun_out -type f -size +4M -print -delete; du -sh gpurun_out' EXIT
timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_conv_wgrad.py tests/test_gpu_consumer.py -k "first_layer or c4 or consumer or disc or patch or fused or dgrad" > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; grep -E "^(FAILED|ERROR)" $O/pytest.log | head; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python scripts/c4w_bench.py --patch-only > $O/c4w_bench.jsonl 2>&1 || { tail -20 $O/c4w_bench.jsonl; exit 1; }
grep c4p $O/c4w_bench.jsonl
for i in 1 2 3; do
  timeout -k 10 200 python bench.py --consumer disc --steps 2000 > $O/disc.log 2>&1 || { tail -5 $O/disc.log; exit 1; }
  grep '^{' $O/disc.log | tee -a $O/disc_default.jsonl | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'disc':d['value'],'ms':d['ms_per_step']}))"
done
bash scripts/gpurun/disc_trace.sh r6b11 > /dev/null || exit 1
cp gpurun_out/trace_r6b11/step_sequence.txt $O/disc_step_sequence.txt
grep -A19 "mean over" $O/disc_step_sequence.txt | head -20
