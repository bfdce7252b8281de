#!/bin/bash
# GPU session 4: tile-variant tests (4 LDS-DMA stages), disc bench sweep over conv staging / tiles, traces.
set -u
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
export TMPDIR=/tmp
trap 'find gpurun_out -type f -size +4M -print -delete; du -sh gpurun_out' EXIT
timeout -k 10 500 python -u -m pytest -x -q --timeout 150 --timeout-method thread -p no:cacheprovider \
  tests/test_conv_wgrad.py -m gpu -k "tile_variants or patch_forward" > gpurun_out/b4_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/b4_pytest.log; grep -E "^(FAILED|E  )" gpurun_out/b4_pytest.log | head -20; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for v in "X=0" "BT_CONV1_TILES=-1" "BT_CONV1_TILES=2" "BT_CONV1_TILES=8" "BT_CONV1_ROWS=4" "BT_CONV_STAGING=3" "BT_CONV_STAGING=4" "BT_CONV_BM=64" "BT_CONV_DGRAD_CLS=1" "BT_WGRAD_STAGING=3" "X=0"; do
  timeout -k 10 200 env $v python bench.py --consumer disc --steps 2000 > gpurun_out/sweep4.log 2>&1 || { tail -5 gpurun_out/sweep4.log; exit 1; }
  grep '^{' gpurun_out/sweep4.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'v':'$v','value':d['value'],'ms':d['ms_per_step']}))" | tee -a gpurun_out/sweep4.jsonl
done
bash scripts/gpurun/disc_trace.sh r4e > /dev/null || exit 1
grep -A30 'per kernel, summed' gpurun_out/trace_r4e/step_sequence.txt
