#!/bin/bash
# Round 6, GPU session 3: 128-channel weight-gradient tiles (tests, per-layer bench, disc A/B),
# the decoded-patch first-layer weight gradient at 4 rows per band (new default), the 1-rank
# RCCL disc step with the graph self-check on a temporary communicator, and a disc step trace.
set -u
cd "$(dirname "$0")/../.."
O=gpurun_out/r6b3
mkdir -p $O
export TMPDIR=/tmp
trap 'find gpurun_out -type f -size +4M -print -delete; du -sh gpurun_out' EXIT
timeout -k 10 400 python -u -m pytest -q --timeout 150 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_conv_wgrad.py tests/test_gpu_consumer.py > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; grep -E "^(FAILED|ERROR)" $O/pytest.log | head -20
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 200 python scripts/wgrad_tiles_bench.py > $O/wgrad_tiles.jsonl 2>&1 || { tail -20 $O/wgrad_tiles.jsonl; exit 1; }
cat $O/wgrad_tiles.jsonl
for v in "co64:" "co128:BT_WGRAD_CO128=1" "co64:" "co128:BT_WGRAD_CO128=1"; do
  name=${v%%:*}; e=${v#*:}
  timeout -k 10 200 env $e python bench.py --consumer disc --steps 2000 > $O/disc.log 2>&1 || { tail -5 $O/disc.log; exit 1; }
  grep '^{' $O/disc.log | tee -a $O/disc_$name.jsonl | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'v':'$name','disc':d['value'],'ms':d['ms_per_step']}))"
done
for v in "temp:" "none:BT_SELFCHECK_GRAPH=0"; do
  name=${v%%:*}; e=${v#*:}
  timeout -k 10 300 env $e python bench.py --consumer disc --force-pg --steps 1000 > $O/disc_pg1.log 2>&1 || { tail -20 $O/disc_pg1.log; exit 1; }
  grep '^{' $O/disc_pg1.log | tee -a $O/disc_pg1_$name.jsonl | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'v':'$name','pg1':d['value'],'sc':d['allreduce_check'].get('selfcheck')}))"
done
bash scripts/gpurun/disc_trace.sh r6b3 > /dev/null || exit 1
cp gpurun_out/trace_r6b3/step_sequence.txt $O/disc_step_sequence.txt
grep -A24 "mean over" $O/disc_step_sequence.txt | head -30
BT_WGRAD_CO128=1 bash scripts/gpurun/disc_trace.sh r6b3c > /dev/null || exit 1
cp gpurun_out/trace_r6b3c/step_sequence.txt $O/disc_step_sequence_co128.txt
grep -A24 "mean over" $O/disc_step_sequence_co128.txt | head -30
