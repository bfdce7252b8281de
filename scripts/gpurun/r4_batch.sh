#!/bin/bash
# One GPU session: consumer tests + smoke + disc bench, new tests, disc trace, DP A/B, densityopt.
set -u
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
export TMPDIR=/tmp
bash scripts/gpurun/quick.sh || exit 1
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_consumer.py tests/test_gpu_loader.py -k "layout or ring_rebuilt or rccl_direct" > gpurun_out/pytest_new3.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_new3.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
bash scripts/gpurun/disc_trace.sh r4b || exit 1
for v in "X=0" "X=0 --force-pg" "X=0 --force-pg --grad-overlap off"; do
  e=${v%% *}; a=""; [ "$e" != "$v" ] && a=${v#* }
  timeout -k 10 200 env $e python bench.py --consumer disc --steps 2000 $a > gpurun_out/dp_ab.log 2>&1 || { tail -5 gpurun_out/dp_ab.log; exit 1; }
  grep '^{' gpurun_out/dp_ab.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'v':'$v','value':d['value'],'ms':d['ms_per_step'],'coll':d['config']['consumer_collectives_per_step'],'order':d['config'].get('grad_buckets_issue_order')}))" | tee -a gpurun_out/dp_ab.jsonl
done
bash scripts/gpurun/dopt_steady.sh
BT_THREAD_REPORT=1 timeout -k 10 200 python bench.py --steps 2000 > gpurun_out/headline.log 2>&1 || { tail -5 gpurun_out/headline.log; exit 1; }
grep '^{' gpurun_out/headline.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'value':d['value'],'ms':d['ms_per_step'],'producers':d['config']['producers_per_gpu'],'cpu':d['cpu']}))"
find gpurun_out -type f -size +4M -print -delete; du -sh gpurun_out
