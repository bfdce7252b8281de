#!/bin/bash
# Round 5: which producer-side BN apply changes the u8-vs-bf16 disc loss
# (test_first_layer_reads_raw_u8_frames_through_decode_table): each variant
# alone, and the two exact on/off comparisons.  A test failure (rc 1) moves on;
# any other exit status ends the script.
set -u
cd "$(dirname "$0")/../.."
O=gpurun_out/r5d13
mkdir -p $O
export TMPDIR=/tmp
run() {
  local name=$1; shift
  timeout -k 10 240 env "$@" python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
    tests/test_conv_wgrad.py -m gpu -k "$K" > $O/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc: $(tail -1 $O/$name.log)"
  grep -E "^E  .*(Expected|Absolute|Mismatch|Greatest|assert)" $O/$name.log | head -6
  [ $rc -le 1 ] || exit $rc
}
K="reads_raw_u8 and c4wave"
run both BT_DUMMY=1
run noconv1 BT_CONV1_BN=0
run noout BT_CONV_OUT_BN=0
run none BT_CONV1_BN=0 BT_CONV_OUT_BN=0
run nohead BT_HEAD_BN_BWD=0
K="applies_its"
run exact BT_DUMMY=1
