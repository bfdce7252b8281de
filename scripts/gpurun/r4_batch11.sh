#!/bin/bash
# GPU session 11 (batches 9 + 10 in one call): new kernels' tests, disc A/B + trace, smoke, headline with
# per-thread CPU, densityopt (4 seeds + steady state); the rest of the GPU suite last.
set -u
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out/b11
export TMPDIR=/tmp
trap 'find gpurun_out -type f -size +4M -print -delete; du -sh gpurun_out' EXIT
timeout -k 10 400 python -u -m pytest -x -q --timeout 150 --timeout-method thread -p no:cacheprovider \
  tests/test_conv_wgrad.py tests/test_gpu_consumer.py -m gpu > gpurun_out/b11/pytest_conv.log 2>&1
rc=$?; tail -2 gpurun_out/b11/pytest_conv.log; grep -E "^(FAILED|E  )" gpurun_out/b11/pytest_conv.log | head -20; [ $rc -eq 0 ] || exit $rc
for v in "X=0" "BT_WGRAD_PIPE=1" "BT_DGRAD_PATCH=0" "BT_C4_DECODED=1" "X=1"; do
  timeout -k 10 200 env $v python bench.py --consumer disc --steps 2000 > gpurun_out/b11/sweep.log 2>&1 || { tail -5 gpurun_out/b11/sweep.log; exit 1; }
  grep '^{' gpurun_out/b11/sweep.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'v':'$v','value':d['value'],'ms':d['ms_per_step']}))" | tee -a gpurun_out/b11/sweep.jsonl
done
bash scripts/gpurun/disc_trace.sh r4k > /dev/null || exit 1
cp gpurun_out/trace_r4k/step_sequence.txt gpurun_out/b11/
sed -n '/mean over/,$p' gpurun_out/trace_r4k/step_sequence.txt | head -40
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/b11/smoke.log 2>&1 || { tail -5 gpurun_out/b11/smoke.log; exit 1; }
tail -2 gpurun_out/b11/smoke.log
timeout -k 10 300 env BT_THREAD_REPORT=1 python bench.py --steps 2000 > gpurun_out/b11/headline.log 2>&1 || { tail -5 gpurun_out/b11/headline.log; exit 1; }
grep '^{' gpurun_out/b11/headline.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({k: d.get(k) for k in ('value','ms_per_step','cpu')}))"
bash scripts/gpurun/dopt_r4.sh || exit 1
timeout -k 10 700 python -u -m pytest -q --timeout 150 --timeout-method thread -p no:cacheprovider tests -m gpu \
  --deselect tests/test_conv_wgrad.py --deselect tests/test_gpu_consumer.py > gpurun_out/b11/pytest_rest.log 2>&1
tail -3 gpurun_out/b11/pytest_rest.log; grep -E "^(FAILED|ERROR)" gpurun_out/b11/pytest_rest.log | head -20
