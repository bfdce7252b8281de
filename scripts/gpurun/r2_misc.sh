#!/bin/bash
# replay kernel numerics + timing (wall and kernel), then the loader-depth A/B
set -u
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
export TMPDIR=/tmp
trap 'find gpurun_out -type f -size +8M -delete' EXIT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_replay.py > gpurun_out/replay_tests.log 2>&1; rc=$?
tail -2 gpurun_out/replay_tests.log; [ $rc -eq 0 ] || { grep -B5 Error gpurun_out/replay_tests.log | head -30; exit $rc; }
bash scripts/gpu_round.sh replay2 rtrace || exit $?
bash scripts/gpurun/r2_prefetch_ab.sh
