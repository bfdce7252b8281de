#!/bin/bash
# densityopt: the reference's 70-epoch run and a 2000-epoch steady-state run with per-phase times
set -u
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out/dopt_r4
timeout -k 10 200 python examples/densityopt/densityopt.py --num-epochs 70 --out-dir gpurun_out/dopt_r4/e70 \
  --json gpurun_out/dopt_r4/e70.json > gpurun_out/dopt_r4/e70.log 2>&1 || { tail -5 gpurun_out/dopt_r4/e70.log; exit 1; }
tail -1 gpurun_out/dopt_r4/e70.log | cut -c1-400
timeout -k 10 300 python examples/densityopt/densityopt.py --num-epochs 2000 --out-dir gpurun_out/dopt_r4/e2000 \
  --image-every 0 --json gpurun_out/dopt_r4/e2000.json > gpurun_out/dopt_r4/e2000.log 2>&1 || { tail -5 gpurun_out/dopt_r4/e2000.log; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/dopt_r4/e2000.json')); print(json.dumps({k: d[k] for k in ('iterations_per_s','abs_diff','steady','d_steps','s_steps')}))"
