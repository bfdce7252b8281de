#!/bin/bash
# GPU session 27: loader without E_AGAIN exceptions (try_recv) -- GPU loader tests,
# then blocking completion waits (BT_LOADER_BLOCKING=1) A/B, disc per-thread CPU.
set -u
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out/b27
export TMPDIR=/tmp
trap 'find gpurun_out -type f -size +4M -print -delete; du -sh gpurun_out' EXIT
timeout -k 10 600 python -u -m pytest -x -q --timeout 150 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_loader.py tests/test_gpu_ownership.py -m gpu > gpurun_out/b27/pytest.log 2>&1
rc=$?; tail -2 gpurun_out/b27/pytest.log; grep -E "^(FAILED|E  )" gpurun_out/b27/pytest.log | head -20; [ $rc -eq 0 ] || exit $rc
for v in "X=0" "BT_LOADER_BLOCKING=1" "X=0" "BT_LOADER_BLOCKING=1"; do
  timeout -k 10 240 env BT_THREAD_REPORT=1 BT_LOADER_CPU=1 $v python bench.py --steps 2000 > gpurun_out/b27/headline.log 2>&1 || { tail -5 gpurun_out/b27/headline.log; exit 1; }
  grep '^{' gpurun_out/b27/headline.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); c=d.get('cpu',{}); print(json.dumps({'v':'$v','value':d['value'],'per':c.get('us_per_frame'),'loader':c.get('loader_us_per_frame'),'thr':c.get('threads_cpu_s')}))" | tee -a gpurun_out/b27/headline.jsonl
done
timeout -k 10 240 env BT_THREAD_REPORT=1 BT_LOADER_CPU=1 python bench.py --consumer disc --steps 2000 > gpurun_out/b27/disc.log 2>&1 || { tail -5 gpurun_out/b27/disc.log; exit 1; }
grep '^{' gpurun_out/b27/disc.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); c=d.get('cpu',{}); print(json.dumps({'v':'disc','value':d['value'],'per':c.get('us_per_frame'),'loader':c.get('loader_us_per_frame'),'thr':c.get('threads_cpu_s')}))" | tee -a gpurun_out/b27/headline.jsonl
