#!/bin/bash
# Round 5, GPU session 6: weight gradients on a side stream, concurrent with
# the data-gradient chain (A/B against the in-line order) and a step trace.
set -u
cd "$(dirname "$0")/../.."
O=gpurun_out/r5b6
mkdir -p $O
export TMPDIR=/tmp
trap 'find gpurun_out -type f -size +4M -print -delete; du -sh gpurun_out' EXIT
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_conv_wgrad.py tests/test_gpu_consumer.py -m gpu > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for v in "side:" "inline:BT_WGRAD_SIDE=0" "side:" "inline:BT_WGRAD_SIDE=0"; do
  name=${v%%:*}; e=${v#*:}
  timeout -k 10 200 env $e python bench.py --consumer disc --steps 2000 > $O/disc.log 2>&1 || { tail -5 $O/disc.log; exit 1; }
  grep '^{' $O/disc.log | tee -a $O/disc_$name.jsonl | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'v':'$name','disc':d['value'],'ms':d['ms_per_step']}))"
done
bash scripts/gpurun/disc_trace.sh r5b6 > /dev/null || exit 1
cp gpurun_out/trace_r5b6/step_sequence.txt $O/disc_step_sequence.txt
grep -A26 "mean over" $O/disc_step_sequence.txt
for v in "st:" "nt:BT_REPLAY_NT=1" "st:" "nt:BT_REPLAY_NT=1"; do
  name=${v%%:*}; e=${v#*:}
  timeout -k 10 120 env $e python benchmarks/bench_replay.py --batch 64 --steps 2000 > $O/replay.log 2>&1 || { tail -5 $O/replay.log; exit 1; }
  grep '^{' $O/replay.log | tee -a $O/replay_$name.jsonl | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'v':'$name','us':d['us_per_batch'],'tbps':d['effective_tbps']}))"
done
timeout -k 10 120 python scripts/bn_apply_bench.py > $O/bn_apply_bench.jsonl 2>&1 || { tail -5 $O/bn_apply_bench.jsonl; exit 1; }
timeout -k 10 120 env BT_BN_RELEASE=0 python scripts/bn_apply_bench.py >> $O/bn_apply_bench.jsonl 2>&1 || { tail -5 $O/bn_apply_bench.jsonl; exit 1; }
cat $O/bn_apply_bench.jsonl
timeout -k 10 300 python scripts/c4w_bench.py --iters 200 > $O/c4w_bench.jsonl 2>&1 || { tail -5 $O/c4w_bench.jsonl; exit 1; }
grep '"waves": 4, "target_blocks": 512' $O/c4w_bench.jsonl
