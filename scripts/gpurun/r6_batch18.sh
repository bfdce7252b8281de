#!/bin/bash
# Round 6, GPU session 18: the lean head forward's per-wave partial logits (one wait with its BN adds)
# and its last block's BN-sum tail with 8 images' loads in flight: GPU suite, disc x3 + trace,
# densityopt steady + trace.
set -u
cd "$(dirname "$0")/../.."
O=gpurun_out/r6b18
mkdir -p $O
export TMPDIR=/tmp
trap 'find gpurun_out -type f -size +4M -print -delete; du -sh gpurun_out' EXIT
timeout -k 10 700 python -u -m pytest -q --timeout 150 --timeout-method thread -p no:cacheprovider -m gpu tests \
  > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; grep -E "^(FAILED|ERROR)" $O/pytest.log | head -20
[ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do
  timeout -k 10 200 python bench.py --consumer disc --steps 2000 > $O/disc.log 2>&1 || { tail -5 $O/disc.log; exit 1; }
  grep '^{' $O/disc.log | tee -a $O/disc_default.jsonl | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'disc':d['value'],'ms':d['ms_per_step']}))"
done
bash scripts/gpurun/disc_trace.sh r6b18 > /dev/null || exit 1
cp gpurun_out/trace_r6b18/step_sequence.txt $O/disc_step_sequence.txt
grep -A19 "mean over" $O/disc_step_sequence.txt | head -20; head -1 $O/disc_step_sequence.txt
timeout -k 10 240 rocprofv3 --kernel-trace -d /tmp/dtr_dopt -o run --output-format csv -- python examples/densityopt/densityopt.py --num-epochs 400 --image-every 0 --out-dir '' > $O/dopt_trace.log 2>&1 || { tail -5 $O/dopt_trace.log; exit 1; }
python scripts/dopt_iteration.py /tmp/dtr_dopt --iters 200 > $O/dopt_iteration_kernels.txt || exit 1
head -12 $O/dopt_iteration_kernels.txt
