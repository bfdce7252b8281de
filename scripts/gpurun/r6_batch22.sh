#!/bin/bash
# Round 6, GPU session 22 (validation after the update took the last slice reduce): whole GPU suite,
# smoke(), headline bench (2000 steps + 20), disc x3, densityopt (steady, trace, 70 epochs x 4
# seeds), the disc roofline with PMC.
set -u
cd "$(dirname "$0")/../.."
O=gpurun_out/r6b22
mkdir -p $O
export TMPDIR=/tmp
trap 'find gpurun_out -type f -size +4M -print -delete; du -sh gpurun_out' EXIT
timeout -k 10 900 python -u -m pytest -q --timeout 200 --timeout-method thread -p no:cacheprovider tests -m gpu \
  > $O/pytest_gpu.log 2>&1
rc=$?; tail -3 $O/pytest_gpu.log; grep -E "^(FAILED|ERROR)" $O/pytest_gpu.log | head -20
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python bench.py > $O/bench_default.log 2>&1 || { tail -5 $O/bench_default.log; exit 1; }
grep '^{' $O/bench_default.log | tee $O/bench_default.jsonl | cut -c1-160
timeout -k 10 300 python bench.py --steps 20 --warmup 10 > $O/bench_20.log 2>&1 || { tail -5 $O/bench_20.log; exit 1; }
grep '^{' $O/bench_20.log | tee $O/bench_20.jsonl | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'v20':d['value'],'sustained':d['sustained']['images_per_s']}))"
for i in 1 2 3; do
  timeout -k 10 200 python bench.py --consumer disc --steps 2000 > $O/disc.log 2>&1 || { tail -5 $O/disc.log; exit 1; }
  grep '^{' $O/disc.log | tee -a $O/disc_default.jsonl | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'disc':d['value'],'ms':d['ms_per_step']}))"
done
timeout -k 10 300 python examples/densityopt/densityopt.py --num-epochs 2000 --image-every 0 --out-dir '' \
  --json $O/dopt_steady.json > $O/dopt_steady.log 2>&1 || { tail -5 $O/dopt_steady.log; exit 1; }
python -c "import json; d=json.load(open('$O/dopt_steady.json')); print(json.dumps({'it_s':round(d['iterations_per_s'],1),'steady':d['steady']['iterations_per_s'],'gpu_it':d['steady']['ms_per_iteration']['gpu_iteration']}))"
timeout -k 10 240 rocprofv3 --kernel-trace -d /tmp/dtr_dopt -o run --output-format csv -- python examples/densityopt/densityopt.py --num-epochs 400 --image-every 0 --out-dir '' > $O/dopt_trace.log 2>&1 || { tail -5 $O/dopt_trace.log; exit 1; }
python scripts/dopt_iteration.py /tmp/dtr_dopt --iters 200 > $O/dopt_iteration_kernels.txt || exit 1
head -3 $O/dopt_iteration_kernels.txt
timeout -k 10 300 python examples/densityopt/densityopt.py --num-epochs 70 --num-runs 4 --image-every 0 \
  --out-dir $O/dopt_e70 --json $O/dopt_e70.json > $O/dopt_e70.log 2>&1 || { tail -5 $O/dopt_e70.log; exit 1; }
python -c "
import json; d=json.load(open('$O/dopt_e70.json'))
for r in d.get('runs',[d]): print(json.dumps({'it_s':round(r['iterations_per_s'],1),'abs_diff':[round(x,3) for x in r['abs_diff']]}))"
bash scripts/gpurun/disc_roofline.sh r6b22 > $O/roofline.log 2>&1 || { tail -20 $O/roofline.log; exit 1; }
cp gpurun_out/roof_r6b22/roofline.md gpurun_out/roof_r6b22/step_sequence.txt $O/
head -1 $O/step_sequence.txt; tail -20 $O/roofline.md
