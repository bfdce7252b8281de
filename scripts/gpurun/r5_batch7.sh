#!/bin/bash
# Round 5, GPU session 7: BN apply release after the stores, first-layer weight
# gradient with its table load first, replay non-temporal stores by default,
# conv1 forward without alpha lookups; disc bench, trace and microbenchmarks.
set -u
cd "$(dirname "$0")/../.."
O=gpurun_out/r5b7
mkdir -p $O
export TMPDIR=/tmp
trap 'find gpurun_out -type f -size +4M -print -delete; du -sh gpurun_out' EXIT
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_conv_wgrad.py tests/test_gpu_consumer.py tests/test_gpu_kernels.py tests/test_replay.py -m gpu > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for i in 1 2; do
  timeout -k 10 200 python bench.py --consumer disc --steps 2000 > $O/disc.log 2>&1 || { tail -5 $O/disc.log; exit 1; }
  grep '^{' $O/disc.log | tee -a $O/disc.jsonl | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'disc':d['value'],'ms':d['ms_per_step']}))"
done
bash scripts/gpurun/disc_trace.sh r5b7 > /dev/null || exit 1
cp gpurun_out/trace_r5b7/step_sequence.txt $O/disc_step_sequence.txt
grep -A23 "mean over" $O/disc_step_sequence.txt | head -24
grep "busy\|median step" $O/disc_step_sequence.txt
timeout -k 10 120 python scripts/bn_apply_bench.py > $O/bn_apply_bench.jsonl 2>&1 || { tail -5 $O/bn_apply_bench.jsonl; exit 1; }
cat $O/bn_apply_bench.jsonl
timeout -k 10 300 python scripts/c4w_bench.py --iters 200 > $O/c4w_bench.jsonl 2>&1 || { tail -5 $O/c4w_bench.jsonl; exit 1; }
grep '"waves": 4, "target_blocks": 512' $O/c4w_bench.jsonl
timeout -k 10 120 python benchmarks/bench_replay.py --batch 64 --steps 2000 > $O/replay64.jsonl 2>&1 || { tail -5 $O/replay64.jsonl; exit 1; }
timeout -k 10 120 python benchmarks/bench_replay.py --batch 8 --steps 2000 > $O/replay8.jsonl 2>&1 || { tail -5 $O/replay8.jsonl; exit 1; }
grep -h '^{' $O/replay64.jsonl $O/replay8.jsonl
