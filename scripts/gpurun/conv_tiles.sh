#!/bin/bash
# Tap-GEMM tile sweep (BT_CONV_BM x BT_CONV_BN) on the bench layers, device
# time from graph replays; then a kernel trace of the default tiles.
set -u
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_conv_wgrad.py \
  > gpurun_out/conv_tests.log 2>&1 || { tail -30 gpurun_out/conv_tests.log; exit 1; }
tail -2 gpurun_out/conv_tests.log
for t in 0:0:0 0:0:2 0:0:3 128:64:3 64:64:3 128:128:3 64:128:3; do
  IFS=: read bm bn st <<< "$t"
  BT_CONV_STAGING=$st BT_CONV_BM=$bm BT_CONV_BN=$bn timeout -k 10 200 python scripts/conv_bench.py --iters 400 > gpurun_out/convt_${st}_${bm}_${bn}.log 2>&1 || { tail gpurun_out/convt_${st}_${bm}_${bn}.log; exit 1; }
  grep -h "^{" gpurun_out/convt_${st}_${bm}_${bn}.log | python -c "
import json, sys
for l in sys.stdin:
    d = json.loads(l)
    print('ST=$st BM=$bm BN=$bn', d['layer'], 'fwd', d['mfma_fwd_us'], d['mfma_fwd_stats_us'], 'dgrad', d['mfma_dgrad_us'], 'miopen fwd', d['miopen_fwd_us'], 'dgrad', d['miopen_dgrad_us'], 'wgrad', d['mfma_us_b512'], d['mfma_us_b1024'], d['miopen_us'])
"
done
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/convprof -o conv --output-format csv -- python3 scripts/conv_bench.py --iters 200 > gpurun_out/convprof.log 2>&1 || { tail gpurun_out/convprof.log; exit 1; }
f=$(find gpurun_out/convprof -name "*kernel_stats.csv" | head -1); python - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs']))[:25]:
    print(f"{float(r['AverageNs'])/1e3:9.2f} us  x{r['Calls']:>6}  {r['Name'][:110]}")
PY
