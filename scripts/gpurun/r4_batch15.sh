#!/bin/bash
# GPU session 15: data-gradient patch with one weight buffer (3 blocks per CU), wide slice groups for the first-layer reduce -- conv + consumer tests, A/B, trace.
set -u
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out/b15
export TMPDIR=/tmp
trap 'find gpurun_out -type f -size +4M -print -delete; du -sh gpurun_out' EXIT
timeout -k 10 400 python -u -m pytest -x -q --timeout 150 --timeout-method thread -p no:cacheprovider \
  tests/test_conv_wgrad.py -m gpu -k "dgrad or wgrad or discriminator or bn" > gpurun_out/b15/pytest.log 2>&1
rc=$?; tail -2 gpurun_out/b15/pytest.log; grep -E "^(FAILED|E  )" gpurun_out/b15/pytest.log | head -20; [ $rc -eq 0 ] || exit $rc
for v in "X=0" "BT_DGRAD_PATCH=0" "X=1" "BT_DGRAD_PATCH=0"; do
  timeout -k 10 200 env $v python bench.py --consumer disc --steps 2000 > gpurun_out/b15/sweep.log 2>&1 || { tail -5 gpurun_out/b15/sweep.log; exit 1; }
  grep '^{' gpurun_out/b15/sweep.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'v':'$v','value':d['value'],'ms':d['ms_per_step']}))" | tee -a gpurun_out/b15/sweep.jsonl
done
bash scripts/gpurun/disc_trace.sh r4o > /dev/null || exit 1
cp gpurun_out/trace_r4o/step_sequence.txt gpurun_out/b15/
sed -n '/mean over/,$p' gpurun_out/trace_r4o/step_sequence.txt | head -40
