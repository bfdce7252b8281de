#!/bin/bash
# Round-4 final validation: the whole GPU suite, smoke(), the headline with the
# round's defaults (2000 and 20 steps, per-thread CPU), the disc consumer, a disc
# step trace.
set -u
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out/final2
export TMPDIR=/tmp
trap 'find gpurun_out -type f -size +4M -print -delete; du -sh gpurun_out' EXIT
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final2/smoke.log 2>&1 || { tail -5 gpurun_out/final2/smoke.log; exit 1; }
tail -1 gpurun_out/final2/smoke.log
for st in 2000 20 2000; do
  timeout -k 10 300 env BT_THREAD_REPORT=1 python bench.py --steps $st > gpurun_out/final2/headline.log 2>&1 || { tail -5 gpurun_out/final2/headline.log; exit 1; }
  grep '^{' gpurun_out/final2/headline.log | tee -a gpurun_out/final2/headline.jsonl | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'steps':$st,'value':d['value'],'ms':d['ms_per_step'],'cpu':d.get('cpu',{}).get('us_per_frame')}))"
done
for r in 1 2; do
  timeout -k 10 300 python bench.py --consumer disc --steps 2000 > gpurun_out/final2/disc.log 2>&1 || { tail -5 gpurun_out/final2/disc.log; exit 1; }
  grep '^{' gpurun_out/final2/disc.log | tee -a gpurun_out/final2/disc.jsonl | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'disc':d['value'],'ms':d['ms_per_step']}))"
done
bash scripts/gpurun/disc_trace.sh r4final2 > /dev/null || exit 1
cp gpurun_out/trace_r4final2/step_sequence.txt gpurun_out/final2/disc_step_sequence.txt
head -1 gpurun_out/final2/disc_step_sequence.txt
timeout -k 10 1000 python -u -m pytest -q --timeout 150 --timeout-method thread -p no:cacheprovider tests -m gpu \
  > gpurun_out/final2/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/final2/pytest_gpu.log; grep -E "^(FAILED|ERROR)" gpurun_out/final2/pytest_gpu.log | head -20; exit $rc
