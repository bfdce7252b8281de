#!/bin/bash
# Disc consumer: process group x communicator, same box
set -u
cd "$(dirname "$0")/../.."
for v in "X=0" "X=0 --force-pg" "BT_DEVICECOMM_DEDICATED=0 --force-pg" "X=0 --force-pg --consumer-input resident" "BT_DEVICECOMM_DEDICATED=0 --force-pg --consumer-input resident"; do
  e=${v%% *}; a=""; [ "$e" != "$v" ] && a=${v#* }
  timeout -k 10 200 env $e python bench.py --consumer disc --steps 1500 $a > gpurun_out/disc_ab.log 2>&1 || { tail -5 gpurun_out/disc_ab.log; exit 1; }
  grep '^{' gpurun_out/disc_ab.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', d['value'], d['ms_per_step'])"
done
