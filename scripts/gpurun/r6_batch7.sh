#!/bin/bash
# Round 6, GPU session 7: the split-K forward of the 128- and 256-channel layers (tap_gemm_body
# SPLIT = 2), the first layer's patch decode in 16-byte loads, 8 vectors per lane in the folding
# BN applies: whole GPU suite, per-kernel microbenches, disc A/B.
set -u
cd "$(dirname "$0")/../.."
O=gpurun_out/r6b7
mkdir -p $O
export TMPDIR=/tmp
trap 'find gpurun_out -type f -size +4M -print -delete; du -sh gpurun_out' EXIT
timeout -k 10 700 python -u -m pytest -q --timeout 150 --timeout-method thread -p no:cacheprovider -m gpu tests \
  > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; grep -E "^(FAILED|ERROR)" $O/pytest.log | head -20
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 200 python scripts/fwd_split_bench.py > $O/fwd_split.jsonl 2>&1 || { tail -20 $O/fwd_split.jsonl; exit 1; }
cat $O/fwd_split.jsonl
timeout -k 10 200 python scripts/c4w_bench.py --patch-only > $O/c4w_bench.jsonl 2>&1 || { tail -20 $O/c4w_bench.jsonl; exit 1; }
cat $O/c4w_bench.jsonl
for u in 4 8; do
  timeout -k 10 200 env BT_BN_UNROLL=$u python scripts/bn_apply_bench.py > $O/bn_apply_u$u.jsonl 2>&1 || { tail -20 $O/bn_apply_u$u.jsonl; exit 1; }
  echo "unroll $u"; cat $O/bn_apply_u$u.jsonl
done
for v in "default:" "u4:BT_BN_UNROLL=4" "split:BT_CONV_FWD_SPLIT=1" "default:" "u4:BT_BN_UNROLL=4" "split:BT_CONV_FWD_SPLIT=1"; do
  name=${v%%:*}; e=${v#*:}
  timeout -k 10 200 env $e python bench.py --consumer disc --steps 2000 > $O/disc.log 2>&1 || { tail -5 $O/disc.log; exit 1; }
  grep '^{' $O/disc.log | tee -a $O/disc_$name.jsonl | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'v':'$name','disc':d['value'],'ms':d['ms_per_step']}))"
done
bash scripts/gpurun/disc_trace.sh r6b7 > /dev/null || exit 1
cp gpurun_out/trace_r6b7/step_sequence.txt $O/disc_step_sequence.txt
grep -A24 "mean over" $O/disc_step_sequence.txt | head -30
