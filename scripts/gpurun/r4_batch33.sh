#!/bin/bash
# GPU session 33: BN apply grid -- cap 512 / 384 with even passes per block vs the
# 1024 cap; BN tests under the chosen grid; trace.
set -u
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out/b33
export TMPDIR=/tmp
trap 'find gpurun_out -type f -size +4M -print -delete; du -sh gpurun_out' EXIT
timeout -k 10 400 env BT_BN_FOLD_GRID=512 BT_BN_FOLD_BALANCE=1 python -u -m pytest -x -q --timeout 150 --timeout-method thread \
  -p no:cacheprovider tests/test_gpu_consumer.py tests/test_conv_wgrad.py -m gpu -k "bn or BN or lazy or fold" > gpurun_out/b33/pytest.log 2>&1
rc=$?; tail -2 gpurun_out/b33/pytest.log; grep -E "^(FAILED|E  )" gpurun_out/b33/pytest.log | head -20; [ $rc -eq 0 ] || exit $rc
for v in "X=0" "BT_BN_FOLD_GRID=512 BT_BN_FOLD_BALANCE=1" "BT_BN_FOLD_GRID=384 BT_BN_FOLD_BALANCE=1" "BT_BN_FOLD_GRID=512" \
         "X=0" "BT_BN_FOLD_GRID=512 BT_BN_FOLD_BALANCE=1" "BT_BN_FOLD_GRID=384 BT_BN_FOLD_BALANCE=1" "BT_BN_FOLD_GRID=512"; do
  timeout -k 10 200 env $v python bench.py --consumer disc --steps 2000 > gpurun_out/b33/sweep.log 2>&1 || { tail -5 gpurun_out/b33/sweep.log; exit 1; }
  grep '^{' gpurun_out/b33/sweep.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'v':'$v','value':d['value'],'ms':d['ms_per_step']}))" | tee -a gpurun_out/b33/sweep.jsonl
done
BT_BN_FOLD_GRID=512 BT_BN_FOLD_BALANCE=1 bash scripts/gpurun/disc_trace.sh r4u > /dev/null || exit 1
cp gpurun_out/trace_r4u/step_sequence.txt gpurun_out/b33/
head -1 gpurun_out/b33/step_sequence.txt
grep -A16 "per kernel, summed" gpurun_out/b33/step_sequence.txt | head -18
