#!/bin/bash
# Round 6, GPU session 10: the fused data + weight gradient launch with a 4-deep dY / X ring in its
# 128-channel weight-gradient blocks (BT_WGRAD_CO128_DEPTH=4, 2 waves per SIMD) against depth 2.
set -u
cd "$(dirname "$0")/../.."
O=gpurun_out/r6b10
mkdir -p $O
export TMPDIR=/tmp
trap 'find gpurun_out -type f -size +4M -print -delete; du -sh gpurun_out' EXIT
timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_conv_wgrad.py -k "co128 or fused" > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
BT_WGRAD_CO128_DEPTH=4 timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_conv_wgrad.py -k "co128 or fused" > $O/pytest_d4.log 2>&1
rc=$?; tail -2 $O/pytest_d4.log; [ $rc -eq 0 ] || exit $rc
for d in 2 4; do
  BT_WGRAD_CO128_DEPTH=$d timeout -k 10 200 python scripts/wgrad_tiles_bench.py > $O/wgrad_tiles_d$d.jsonl 2>&1 || { tail -20 $O/wgrad_tiles_d$d.jsonl; exit 1; }
  echo "depth $d"; grep '"co128": 1' $O/wgrad_tiles_d$d.jsonl
done
for v in "default:" "d4:BT_WGRAD_CO128_DEPTH=4" "default:" "d4:BT_WGRAD_CO128_DEPTH=4"; do
  name=${v%%:*}; e=${v#*:}
  timeout -k 10 200 env $e python bench.py --consumer disc --steps 2000 > $O/disc.log 2>&1 || { tail -5 $O/disc.log; exit 1; }
  grep '^{' $O/disc.log | tee -a $O/disc_$name.jsonl | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'v':'$name','disc':d['value'],'ms':d['ms_per_step']}))"
done
