#!/bin/bash
# GPU session 14: data-gradient patch on by default (BN inputs prefetched) -- conv + consumer tests, A/B, trace.
set -u
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out/b14
export TMPDIR=/tmp
trap 'find gpurun_out -type f -size +4M -print -delete; du -sh gpurun_out' EXIT
timeout -k 10 400 python -u -m pytest -x -q --timeout 150 --timeout-method thread -p no:cacheprovider \
  tests/test_conv_wgrad.py tests/test_gpu_consumer.py -m gpu > gpurun_out/b14/pytest.log 2>&1
rc=$?; tail -2 gpurun_out/b14/pytest.log; grep -E "^(FAILED|E  )" gpurun_out/b14/pytest.log | head -20; [ $rc -eq 0 ] || exit $rc
for v in "X=0" "BT_DGRAD_PATCH=0" "X=1" "BT_DGRAD_PATCH=0"; do
  timeout -k 10 200 env $v python bench.py --consumer disc --steps 2000 > gpurun_out/b14/sweep.log 2>&1 || { tail -5 gpurun_out/b14/sweep.log; exit 1; }
  grep '^{' gpurun_out/b14/sweep.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'v':'$v','value':d['value'],'ms':d['ms_per_step']}))" | tee -a gpurun_out/b14/sweep.jsonl
done
bash scripts/gpurun/disc_trace.sh r4n > /dev/null || exit 1
cp gpurun_out/trace_r4n/step_sequence.txt gpurun_out/b14/
sed -n '/mean over/,$p' gpurun_out/trace_r4n/step_sequence.txt | head -40
