#!/bin/bash
# Round 6, GPU session 8: the BN accumulator release's ticket taken after the fold and answered at
# the end of the block (apply launches and the first layer's weight gradient): GPU tests, the apply
# bench (new form vs the whole release before the pass, BT_BN_RELEASE=2), c4p, disc A/B, trace.
set -u
cd "$(dirname "$0")/../.."
O=gpurun_out/r6b8
mkdir -p $O
export TMPDIR=/tmp
trap 'find gpurun_out -type f -size +4M -print -delete; du -sh gpurun_out' EXIT
timeout -k 10 700 python -u -m pytest -q --timeout 150 --timeout-method thread -p no:cacheprovider -m gpu tests \
  > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; grep -E "^(FAILED|ERROR)" $O/pytest.log | head -20
[ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  timeout -k 10 120 env BT_BN_RELEASE=$r python scripts/bn_apply_bench.py > $O/bn_apply_rel$r.jsonl 2>&1 || { tail -20 $O/bn_apply_rel$r.jsonl; exit 1; }
  echo "release $r"; grep '^{' $O/bn_apply_rel$r.jsonl | grep fold
done
timeout -k 10 200 python scripts/c4w_bench.py --patch-only > $O/c4w_bench.jsonl 2>&1 || { tail -20 $O/c4w_bench.jsonl; exit 1; }
grep c4p $O/c4w_bench.jsonl
for v in "default:" "rel2:BT_BN_RELEASE=2" "default:" "rel2:BT_BN_RELEASE=2"; do
  name=${v%%:*}; e=${v#*:}
  timeout -k 10 200 env $e python bench.py --consumer disc --steps 2000 > $O/disc.log 2>&1 || { tail -5 $O/disc.log; exit 1; }
  grep '^{' $O/disc.log | tee -a $O/disc_$name.jsonl | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'v':'$name','disc':d['value'],'ms':d['ms_per_step']}))"
done
bash scripts/gpurun/disc_trace.sh r6b8 > /dev/null || exit 1
cp gpurun_out/trace_r6b8/step_sequence.txt $O/disc_step_sequence.txt
grep -A24 "mean over" $O/disc_step_sequence.txt | head -30
