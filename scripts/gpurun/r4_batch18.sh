#!/bin/bash
# GPU session 18: weight gradient over 256-column tiles (BT_WGRAD_WIDE) -- tests, A/B, trace.
set -u
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out/b18
export TMPDIR=/tmp
trap 'find gpurun_out -type f -size +4M -print -delete; du -sh gpurun_out' EXIT
timeout -k 10 400 python -u -m pytest -x -q --timeout 150 --timeout-method thread -p no:cacheprovider \
  tests/test_conv_wgrad.py -m gpu -k "wgrad" > gpurun_out/b18/pytest.log 2>&1
rc=$?; tail -2 gpurun_out/b18/pytest.log; grep -E "^(FAILED|E  )" gpurun_out/b18/pytest.log | head -20; [ $rc -eq 0 ] || exit $rc
for v in "X=0" "BT_WGRAD_WIDE=1" "X=1" "BT_WGRAD_WIDE=1"; do
  timeout -k 10 200 env $v python bench.py --consumer disc --steps 2000 > gpurun_out/b18/sweep.log 2>&1 || { tail -5 gpurun_out/b18/sweep.log; exit 1; }
  grep '^{' gpurun_out/b18/sweep.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'v':'$v','value':d['value'],'ms':d['ms_per_step']}))" | tee -a gpurun_out/b18/sweep.jsonl
done
BT_WGRAD_WIDE=1 bash scripts/gpurun/disc_trace.sh r4r > /dev/null || exit 1
cp gpurun_out/trace_r4r/step_sequence.txt gpurun_out/b18/
sed -n '/mean over/,/per kernel/p' gpurun_out/trace_r4r/step_sequence.txt | head -26
