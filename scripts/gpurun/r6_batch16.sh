#!/bin/bash
# Round 6, GPU session 16: same-box A/B of the disc step -- this session's start (commit 4fd000a,
# built in ab_old/) against the current tree, alternating, 2000 steps each; the head weight
# gradient's 8 images in flight (densityopt iteration trace, batch 64); the first-layer forward's
# two-tile-ahead prefetch at 4 (1200 blocks) and 5 (960 blocks, all resident at 4 waves per SIMD)
# tiles per block.
set -u
cd "$(dirname "$0")/../.."
O=gpurun_out/r6b16
mkdir -p $O
export TMPDIR=/tmp
trap 'find gpurun_out -type f -size +4M -print -delete; du -sh gpurun_out' EXIT
timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_gpu_consumer.py tests/test_densityopt.py > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; grep -E "^(FAILED|ERROR)" $O/pytest.log | head; [ $rc -eq 0 ] || exit $rc
for v in new old new5 new old new5 new old; do
  e=""; d=.
  [ $v = old ] && d=ab_old
  [ $v = new5 ] && e="BT_CONV1_TILES=5"
  timeout -k 10 200 env $e python $d/bench.py --consumer disc --steps 2000 > $O/disc.log 2>&1 || { tail -5 $O/disc.log; exit 1; }
  grep '^{' $O/disc.log | tee -a $O/disc_$v.jsonl | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'v':'$v','disc':d['value'],'ms':d['ms_per_step']}))"
done
bash scripts/gpurun/disc_trace.sh r6b16 > /dev/null || exit 1
cp gpurun_out/trace_r6b16/step_sequence.txt $O/disc_step_sequence.txt
grep -A19 "mean over" $O/disc_step_sequence.txt | head -20; head -1 $O/disc_step_sequence.txt
timeout -k 10 240 rocprofv3 --kernel-trace -d /tmp/dtr_dopt -o run --output-format csv -- python examples/densityopt/densityopt.py --num-epochs 400 --image-every 0 --out-dir '' > $O/dopt_trace.log 2>&1 || { tail -5 $O/dopt_trace.log; exit 1; }
python scripts/dopt_iteration.py /tmp/dtr_dopt --iters 200 > $O/dopt_iteration_kernels.txt || exit 1
head -14 $O/dopt_iteration_kernels.txt
