#!/bin/bash
# Round 5, GPU session 4: the round-trip-lean head forward, head backward
# loads, conflict-free BN-apply coefficients -- tests, same-call disc A/B,
# step trace; then the per-layer tile / staging sweep.
set -u
cd "$(dirname "$0")/../.."
O=gpurun_out/r5b4
mkdir -p $O
export TMPDIR=/tmp
trap 'find gpurun_out -type f -size +4M -print -delete; du -sh gpurun_out' EXIT
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_consumer.py tests/test_gpu_kernels.py -m gpu > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for v in "new:" "r4head:BT_HEAD_FWD=0" "new:" "r4head:BT_HEAD_FWD=0"; do
  name=${v%%:*}; e=${v#*:}
  timeout -k 10 200 env $e python bench.py --consumer disc --steps 2000 > $O/disc.log 2>&1 || { tail -5 $O/disc.log; exit 1; }
  grep '^{' $O/disc.log | tee -a $O/disc_$name.jsonl | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'v':'$name','disc':d['value'],'ms':d['ms_per_step']}))"
done
bash scripts/gpurun/disc_trace.sh r5b4 > /dev/null || exit 1
cp gpurun_out/trace_r5b4/step_sequence.txt $O/disc_step_sequence.txt
head -26 $O/disc_step_sequence.txt
timeout -k 10 600 python scripts/conv_tile_sweep.py --iters 200 > $O/tile_sweep.jsonl 2>&1 || { tail -5 $O/tile_sweep.jsonl; exit 1; }
grep BEST $O/tile_sweep.jsonl
