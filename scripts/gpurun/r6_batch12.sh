#!/bin/bash
# Round 6, GPU session 12: the patch data gradient back to one class ahead with its BN inputs as
# 16-byte loads issued first; the decode / replay kernels' pixels as 32-bit words (no scratch); the
# folding BN applies' next-pass prefetch (A/B BT_BN_PREFETCH): GPU suite, BN apply bench, disc A/B +
# trace, replay bench (batch 8 / 64, both table forms), headline bench.
set -u
cd "$(dirname "$0")/../.."
O=gpurun_out/r6b12
mkdir -p $O
export TMPDIR=/tmp
trap 'find gpurun_out -type f -size +4M -print -delete; du -sh gpurun_out' EXIT
timeout -k 10 700 python -u -m pytest -q --timeout 150 --timeout-method thread -p no:cacheprovider -m gpu tests \
  > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; grep -E "^(FAILED|ERROR)" $O/pytest.log | head -20
[ $rc -eq 0 ] || exit $rc
for pf in 1 0; do
  BT_BN_PREFETCH=$pf timeout -k 10 120 python scripts/bn_apply_bench.py > $O/bn_apply_pf$pf.jsonl 2>&1 || { tail -20 $O/bn_apply_pf$pf.jsonl; exit 1; }
  echo "prefetch $pf"; grep '"fold"' $O/bn_apply_pf$pf.jsonl
done
for v in "default:" "nopf:BT_BN_PREFETCH=0" "default:" "nopf:BT_BN_PREFETCH=0" "default:"; do
  name=${v%%:*}; e=${v#*:}
  timeout -k 10 200 env $e python bench.py --consumer disc --steps 2000 > $O/disc.log 2>&1 || { tail -5 $O/disc.log; exit 1; }
  grep '^{' $O/disc.log | tee -a $O/disc_$name.jsonl | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'v':'$name','disc':d['value'],'ms':d['ms_per_step']}))"
done
bash scripts/gpurun/disc_trace.sh r6b12 > /dev/null || exit 1
cp gpurun_out/trace_r6b12/step_sequence.txt $O/disc_step_sequence.txt
grep -A19 "mean over" $O/disc_step_sequence.txt | head -20
for x in 0 auto; do
  for args in "--batch 8" "--batch 64 --steps 500"; do
    BLENDTORCH_DECODE_XFORM=$x timeout -k 10 120 python benchmarks/bench_replay.py $args > $O/replay.log 2>&1 || { tail -5 $O/replay.log; exit 1; }
    grep '^{' $O/replay.log | tee -a $O/replay_x$x.jsonl | python -c "
import json,sys
d=json.loads(sys.stdin.read()); print('xform=$x', 'B', d['batch'], d['us_per_batch'], 'us', d['effective_tbps'], 'TB/s')"
  done
done
timeout -k 10 300 python bench.py > $O/bench_default.log 2>&1 || { tail -5 $O/bench_default.log; exit 1; }
grep '^{' $O/bench_default.log | tee $O/bench_default.jsonl | cut -c1-160
