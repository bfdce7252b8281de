#!/bin/bash
# conv tests + conv_bench (default tiles) + PMC summary
set -u
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_conv_wgrad.py > gpurun_out/conv_tests.log 2>&1 || { tail -30 gpurun_out/conv_tests.log; exit 1; }
tail -1 gpurun_out/conv_tests.log
timeout -k 10 200 python scripts/conv_bench.py --iters 400 > gpurun_out/convq.log 2>&1 || { tail gpurun_out/convq.log; exit 1; }
grep -h "^{" gpurun_out/convq.log | python -c "
import json, sys
for l in sys.stdin:
    d = json.loads(l)
    print(d['layer'], 'fwd', d['mfma_fwd_us'], d['mfma_fwd_stats_us'], 'dgrad', d['mfma_dgrad_us'], 'miopen fwd', d['miopen_fwd_us'], 'dgrad', d['miopen_dgrad_us'], 'wgrad', d['mfma_us_b512'], d['mfma_us_b1024'], d['miopen_us'])
"
bash scripts/conv_pmc.sh 2>&1 | grep -v "^('btn::gpu::'"
