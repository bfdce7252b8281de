#!/bin/bash
# densityopt: the reference's 70-epoch run over 4 seeds (Abs.Diff per seed, history files + PNG grids),
# then a 2000-epoch steady-state run with per-phase times.
set -u
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out/dopt_r4b
timeout -k 10 500 python examples/densityopt/densityopt.py --num-epochs 70 --num-runs 4 --image-every 35 \
  --out-dir gpurun_out/dopt_r4b/e70 --json gpurun_out/dopt_r4b/e70.json > gpurun_out/dopt_r4b/e70.log 2>&1 \
  || { tail -5 gpurun_out/dopt_r4b/e70.log; exit 1; }
python -c "
import json; d=json.load(open('gpurun_out/dopt_r4b/e70.json'))
for r in d.get('runs', [d]): print(json.dumps({k: r.get(k) for k in ('seed','abs_diff','iterations_per_s')}))"
timeout -k 10 300 python examples/densityopt/densityopt.py --num-epochs 2000 --out-dir gpurun_out/dopt_r4b/e2000 \
  --image-every 0 --json gpurun_out/dopt_r4b/e2000.json > gpurun_out/dopt_r4b/e2000.log 2>&1 \
  || { tail -5 gpurun_out/dopt_r4b/e2000.log; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/dopt_r4b/e2000.json')); print(json.dumps({k: d.get(k) for k in ('iterations_per_s','abs_diff','steady','d_steps','s_steps')}))"
