#!/bin/bash
# Round 6, GPU session 9: a sweep of the disc step's grid / tile knobs on the current kernels
# (one 2000-step run each, the default three times interleaved).
set -u
cd "$(dirname "$0")/../.."
O=gpurun_out/r6b9
mkdir -p $O
export TMPDIR=/tmp
trap 'find gpurun_out -type f -size +4M -print -delete; du -sh gpurun_out' EXIT
for v in "default:" "div1:BT_WGRAD_CO128_DIV=1" "div4:BT_WGRAD_CO128_DIV=4" "wb768:BT_WGRAD_BLOCKS=768" \
         "default:" "wb384:BT_WGRAD_BLOCKS=384" "bm64b256:BT_CONV_BM64_BELOW=256" "bm64b1024:BT_CONV_BM64_BELOW=1024" \
         "default:" "fold1024:BT_BN_FOLD_GRID=1024" "fold256:BT_BN_FOLD_GRID=256" "c1t2:BT_CONV1_TILES=2" "c1t8:BT_CONV1_TILES=8" "default:"; do
  name=${v%%:*}; e=${v#*:}
  timeout -k 10 200 env $e python bench.py --consumer disc --steps 2000 > $O/disc.log 2>&1 || { tail -5 $O/disc.log; exit 1; }
  grep '^{' $O/disc.log | tee -a $O/disc_$name.jsonl | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'v':'$name','disc':d['value'],'ms':d['ms_per_step']}))"
done
