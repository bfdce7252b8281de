#!/bin/bash
# GPU session 10: full GPU suite, smoke, headline bench (+ per-thread CPU), densityopt (4 seeds + steady state).
set -u
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out/b10
export TMPDIR=/tmp
trap 'find gpurun_out -type f -size +4M -print -delete; du -sh gpurun_out' EXIT
timeout -k 10 900 python -u -m pytest -q --timeout 150 --timeout-method thread -p no:cacheprovider tests -m gpu \
  > gpurun_out/b10/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/b10/pytest_gpu.log; grep -E "^(FAILED|ERROR)" gpurun_out/b10/pytest_gpu.log | head -20
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/b10/smoke.log 2>&1 || { tail -5 gpurun_out/b10/smoke.log; exit 1; }
tail -3 gpurun_out/b10/smoke.log
timeout -k 10 300 env BT_THREAD_REPORT=1 python bench.py --steps 2000 > gpurun_out/b10/headline.log 2>&1 || { tail -5 gpurun_out/b10/headline.log; exit 1; }
grep '^{' gpurun_out/b10/headline.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({k: d.get(k) for k in ('value','ms_per_step','cpu','producers')}))"
timeout -k 10 300 python bench.py --consumer disc --steps 2000 > gpurun_out/b10/disc.log 2>&1 || { tail -5 gpurun_out/b10/disc.log; exit 1; }
grep '^{' gpurun_out/b10/disc.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({k: d.get(k) for k in ('value','ms_per_step')}))"
bash scripts/gpurun/dopt_r4.sh || exit 1
