#!/bin/bash
# GPU session 42: the disc consumer with two steps per graph as the default --
# bench x3, trace (idle between replays), then the whole GPU suite.
set -u
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out/b42
export TMPDIR=/tmp
trap 'find gpurun_out -type f -size +4M -print -delete; du -sh gpurun_out' EXIT
for r in 1 2 3; do
  timeout -k 10 200 python bench.py --consumer disc --steps 2000 > gpurun_out/b42/disc.log 2>&1 || { tail -5 gpurun_out/b42/disc.log; exit 1; }
  grep '^{' gpurun_out/b42/disc.log | tee -a gpurun_out/b42/disc.jsonl | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'disc':d['value'],'ms':d['ms_per_step'],'graph_steps':d['config'].get('graph_steps')}))"
done
bash scripts/gpurun/disc_trace.sh r4x > /dev/null || exit 1
grep -E "steps;|between steps|busy" gpurun_out/trace_r4x/step_sequence.txt | tee gpurun_out/b42/disc_step_gaps.txt
rm -f gpurun_out/trace_r4x/bench.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/b42/smoke.log 2>&1 || { tail -5 gpurun_out/b42/smoke.log; exit 1; }
tail -1 gpurun_out/b42/smoke.log
timeout -k 10 1000 python -u -m pytest -q --timeout 150 --timeout-method thread -p no:cacheprovider tests -m gpu \
  > gpurun_out/b42/pytest_gpu.log 2>&1
rc=$?; tail -2 gpurun_out/b42/pytest_gpu.log; grep -E "^(FAILED|ERROR)" gpurun_out/b42/pytest_gpu.log | head -20; exit $rc
