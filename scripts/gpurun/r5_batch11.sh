#!/bin/bash
# Round 5, GPU session 11: the BN apply block cap (BT_BN_FOLD_GRID) -- fewer
# folding blocks for the small applies -- per apply and on the disc step.
set -u
cd "$(dirname "$0")/../.."
O=gpurun_out/r5b11
mkdir -p $O
export TMPDIR=/tmp
trap 'find gpurun_out -type f -size +4M -print -delete; du -sh gpurun_out' EXIT
for cap in 512 256 128 1024; do
  timeout -k 10 120 env BT_BN_FOLD_GRID=$cap python scripts/bn_apply_bench.py > $O/bn_apply_$cap.jsonl 2>&1 || { tail -5 $O/bn_apply_$cap.jsonl; exit 1; }
  python -c "
import json
rows=[json.loads(l) for l in open('$O/bn_apply_$cap.jsonl') if l.startswith('{')]
print('cap $cap', {r['apply']: r['us'] for r in rows if r['variant'] == 'fold'}, 'sum', round(sum(r['us'] for r in rows if r['variant'] == 'fold'), 2))"
done
for v in "c512:" "c256:BT_BN_FOLD_GRID=256" "c128:BT_BN_FOLD_GRID=128" "c512:" "c256:BT_BN_FOLD_GRID=256" "c128:BT_BN_FOLD_GRID=128"; do
  name=${v%%:*}; e=${v#*:}
  timeout -k 10 200 env $e python bench.py --consumer disc --steps 2000 > $O/disc.log 2>&1 || { tail -5 $O/disc.log; exit 1; }
  grep '^{' $O/disc.log | tee -a $O/disc_$name.jsonl | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'v':'$name','disc':d['value'],'ms':d['ms_per_step']}))"
done
