#!/bin/bash
# GPU session 3: conv/consumer tests, disc trace, disc DP A/B at the default queues, smoke.
set -u
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
export TMPDIR=/tmp
trap 'find gpurun_out -type f -size +4M -print -delete; du -sh gpurun_out' EXIT
timeout -k 10 500 python -u -m pytest -x -q --timeout 150 --timeout-method thread -p no:cacheprovider \
  tests/test_conv_wgrad.py tests/test_gpu_consumer.py -m gpu > gpurun_out/b3_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/b3_pytest.log; grep -E "^(FAILED|E  )" gpurun_out/b3_pytest.log | head -20; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
bash scripts/gpurun/disc_trace.sh r4d || exit 1
for v in "X=0" "X=0 --force-pg" "BT_C4_WAVE=0"; do
  e=${v%% *}; a=""; [ "$e" != "$v" ] && a=${v#* }
  timeout -k 10 200 env $e python bench.py --consumer disc --steps 2000 $a > gpurun_out/dp_ab3.log 2>&1 || { tail -5 gpurun_out/dp_ab3.log; exit 1; }
  grep '^{' gpurun_out/dp_ab3.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'v':'$v','value':d['value'],'ms':d['ms_per_step'],'coll':d['config']['consumer_collectives_per_step'],'hwq':d.get('hw_queues')}))" | tee -a gpurun_out/dp_ab3.jsonl
done
timeout -k 10 240 python -c "import sys; sys.path.insert(0,'.'); import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; tail -1 gpurun_out/smoke.log
