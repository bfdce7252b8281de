#!/bin/bash
# GPU session 7: consumer + conv tests (head backward rewrite, BN apply in the head), disc bench, kernel trace.
set -u
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
export TMPDIR=/tmp
trap 'find gpurun_out -type f -size +4M -print -delete; du -sh gpurun_out' EXIT
timeout -k 10 600 python -u -m pytest -x -q --timeout 150 --timeout-method thread -p no:cacheprovider \
  tests/test_conv_wgrad.py::test_forward_applies_input_bn tests/test_conv_wgrad.py::test_wgrad_applies_bn_backward_folded tests/test_gpu_consumer.py tests/test_conv_wgrad.py -m gpu > gpurun_out/b7_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/b7_pytest.log; grep -E "^(FAILED|E  )" gpurun_out/b7_pytest.log | head -20; [ $rc -eq 0 ] || exit $rc
for v in "X=0" "X=1"; do
  timeout -k 10 200 env $v python bench.py --consumer disc --steps 2000 > gpurun_out/sweep7.log 2>&1 || { tail -5 gpurun_out/sweep7.log; exit 1; }
  grep '^{' gpurun_out/sweep7.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'v':'$v','value':d['value'],'ms':d['ms_per_step']}))" | tee -a gpurun_out/sweep7.jsonl
done
bash scripts/gpurun/disc_trace.sh r4h > /dev/null || exit 1
grep -A30 'per kernel, summed' gpurun_out/trace_r4h/step_sequence.txt
# per-kernel effect of the staging depth and the weight-gradient block count
for v in BT_CONV_STAGING=3 BT_CONV_STAGING=4 BT_WGRAD_BLOCKS=1024 BT_WGRAD_BLOCKS=2048; do
  tag=r4h_${v/=/_}
  env $v bash scripts/gpurun/disc_trace.sh $tag > /dev/null || exit 1
  echo "== $v"; grep -A24 'mean over' gpurun_out/trace_$tag/step_sequence.txt
done
