#!/bin/bash
# Round 5, GPU session 2: disc roofline (trace + PMC), densityopt 70 epochs x 4
# seeds (rate beside accuracy) and its iteration's kernel trace, the whole GPU
# suite.
set -u
cd "$(dirname "$0")/../.."
O=gpurun_out/r5b2
mkdir -p $O
export TMPDIR=/tmp
trap 'find gpurun_out -type f -size +4M -print -delete; du -sh gpurun_out' EXIT
bash scripts/gpurun/disc_roofline.sh r5a > $O/roofline_stdout.txt 2>&1 || { tail -20 $O/roofline_stdout.txt; exit 1; }
tail -26 $O/roofline_stdout.txt
timeout -k 10 300 python examples/densityopt/densityopt.py --num-epochs 70 --num-runs 4 --image-every 0 \
  --out-dir $O/dopt_e70 --json $O/dopt_e70.json > $O/dopt_e70.log 2>&1 || { tail -5 $O/dopt_e70.log; exit 1; }
python -c "
import json; d=json.load(open('$O/dopt_e70.json'))
for r in d.get('runs',[d]): print(json.dumps({'it_s':round(r['iterations_per_s'],1),'steady':round(r['steady']['iterations_per_s'],1),'abs_diff':[round(x,3) for x in r['abs_diff']]}))"
timeout -k 10 240 rocprofv3 --kernel-trace -d /tmp/dtr_dopt -o run --output-format csv -- python examples/densityopt/densityopt.py --num-epochs 400 --image-every 0 --out-dir '' > $O/dopt_trace.log 2>&1 || { tail -5 $O/dopt_trace.log; exit 1; }
python scripts/kernel_summary.py /tmp/dtr_dopt --iters 401 > $O/dopt_iteration_kernels.txt || exit 1
head -60 $O/dopt_iteration_kernels.txt
timeout -k 10 1000 python -u -m pytest -q --timeout 150 --timeout-method thread -p no:cacheprovider tests -m gpu \
  > $O/pytest_gpu.log 2>&1
rc=$?; tail -3 $O/pytest_gpu.log; grep -E "^(FAILED|ERROR)" $O/pytest_gpu.log | head -20; exit $rc
