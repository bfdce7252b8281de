#!/bin/bash
# Quick GPU check after a kernel change: the BN / conv / consumer GPU tests, smoke, and a short disc bench.
# Usage: quick.sh [pytest -k expression]
set -u
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
export TMPDIR=/tmp
K=${1:-}
if [ -n "$K" ]; then
  timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
    tests/test_conv_wgrad.py tests/test_gpu_consumer.py tests/test_gpu_kernels.py tests/test_gpu_ownership.py tests/test_models.py tests/test_adam.py -m gpu -k "$K" > gpurun_out/quick_pytest.log 2>&1
else
  timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
    tests/test_conv_wgrad.py tests/test_gpu_consumer.py tests/test_gpu_kernels.py tests/test_gpu_ownership.py tests/test_models.py tests/test_adam.py -m gpu > gpurun_out/quick_pytest.log 2>&1
fi
rc=$?; tail -3 gpurun_out/quick_pytest.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 240 python -c "import sys; sys.path.insert(0,'.'); import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -5 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 200 python bench.py --consumer disc --steps 2000 > gpurun_out/quick_disc.log 2>&1 || { tail -5 gpurun_out/quick_disc.log; exit 1; }
grep '^{' gpurun_out/quick_disc.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('disc', d['value'], d['ms_per_step'], d['config']['consumer_step'])"
