#!/bin/bash
# GPU session 9: channel-tile LDS swizzle (bkey), pipelined weight gradient, 32-channel data gradient from a dY patch -- conv numerics, disc bench, trace, PMC pass 1.
set -u
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
export TMPDIR=/tmp
trap 'find gpurun_out -type f -size +4M -print -delete; du -sh gpurun_out' EXIT
timeout -k 10 600 python -u -m pytest -x -q --timeout 150 --timeout-method thread -p no:cacheprovider \
  tests/test_conv_wgrad.py tests/test_gpu_consumer.py -m gpu > gpurun_out/b9_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/b9_pytest.log; grep -E "^(FAILED|E  )" gpurun_out/b9_pytest.log | head -20; [ $rc -eq 0 ] || exit $rc
for v in "X=0" "BT_WGRAD_PIPE=1" "BT_DGRAD_PATCH=0" "X=1" "BT_WGRAD_PIPE=1"; do
  timeout -k 10 200 env $v python bench.py --consumer disc --steps 2000 > gpurun_out/sweep9.log 2>&1 || { tail -5 gpurun_out/sweep9.log; exit 1; }
  grep '^{' gpurun_out/sweep9.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'v':'$v','value':d['value'],'ms':d['ms_per_step']}))" | tee -a gpurun_out/sweep9.jsonl
done
bash scripts/gpurun/disc_trace.sh r4j > /dev/null || exit 1
sed -n '/mean over/,$p' gpurun_out/trace_r4j/step_sequence.txt | head -40
BT_WGRAD_PIPE=1 bash scripts/gpurun/disc_trace.sh r4j_pipe > /dev/null || exit 1
sed -n '/mean over/,$p' gpurun_out/trace_r4j_pipe/step_sequence.txt | head -30
bash scripts/gpurun/disc_pmc.sh > /dev/null || exit 1
cat gpurun_out/disc_pmc/summary.txt
