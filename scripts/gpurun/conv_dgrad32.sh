#!/bin/bash
# 32-output-channel data gradient (the first BN-fed layer): tile height x staging sweep
set -u
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
for t in 0:0:2 0:0:0 0:0:3 64:0:2 64:0:0 64:0:3 128:0:3; do
  IFS=: read bm bn st <<< "$t"
  BT_CONV_STAGING=$st BT_CONV_BM=$bm BT_CONV_BN=$bn timeout -k 10 200 python scripts/conv_bench.py --iters 400 > gpurun_out/cd32_${st}_${bm}.log 2>&1 || { tail gpurun_out/cd32_${st}_${bm}.log; exit 1; }
  grep -h "^{" gpurun_out/cd32_${st}_${bm}.log | python -c "
import json, sys
for l in sys.stdin:
    d = json.loads(l)
    print('ST=$st BM=$bm', d['layer'], 'fwd', d['mfma_fwd_us'], 'dgrad', d['mfma_dgrad_us'])
"
done
