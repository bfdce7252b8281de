#!/bin/bash
# GPU session 38: two training steps per graph replay (CapturedStep(pair_steps)) --
# the consumer-step tests, smoke, then the disc A/B.
set -u
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out/b38
export TMPDIR=/tmp
trap 'find gpurun_out -type f -size +4M -print -delete; du -sh gpurun_out' EXIT
timeout -k 10 500 python -u -m pytest -x -q --timeout 150 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_consumer.py -m gpu > gpurun_out/b38/pytest.log 2>&1
rc=$?; tail -2 gpurun_out/b38/pytest.log; grep -E "^(FAILED|E  )" gpurun_out/b38/pytest.log | head -20; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/b38/smoke.log 2>&1 || { tail -5 gpurun_out/b38/smoke.log; exit 1; }
tail -1 gpurun_out/b38/smoke.log
for v in "--graph-steps 1" "--graph-steps 2" "--graph-steps 1" "--graph-steps 2" "--graph-steps 1" "--graph-steps 2"; do
  timeout -k 10 200 python bench.py --consumer disc --steps 2000 $v > gpurun_out/b38/sweep.log 2>&1 || { tail -5 gpurun_out/b38/sweep.log; exit 1; }
  grep '^{' gpurun_out/b38/sweep.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'v':'$v','value':d['value'],'ms':d['ms_per_step']}))" | tee -a gpurun_out/b38/sweep.jsonl
done
