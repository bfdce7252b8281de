#!/bin/bash
# Tap-GEMM tile-height sweep (BT_CONV_BM=128 / 64) on the bench layers, after
# the conv/consumer GPU tests; then scatter vs shard on one rank.
set -u
cd "$(dirname "$0")/../.."
bash scripts/gpu_round.sh "gtests:tests/test_conv_wgrad.py,tests/test_gpu_consumer.py,tests/test_gpu_loader.py" || exit $?
for bm in 128 64; do
  BT_CONV_BM=$bm timeout -k 10 200 python scripts/conv_bench.py --iters 200 > gpurun_out/convbm_$bm.log 2>&1 || exit 1
  grep -h "^{" gpurun_out/convbm_$bm.log | python -c "
import json, sys
for l in sys.stdin:
    d = json.loads(l)
    print('BM=$bm', d['layer'], 'fwd', d['mfma_fwd_us'], d['mfma_fwd_stats_us'], 'dgrad', d['mfma_dgrad_us'])
"
done
bash scripts/gpu_round.sh "b:--dist,scatter,--force-pg,--steps,2000" "b:--force-pg,--steps,2000"
