#!/bin/bash
# Round 6, GPU session 2: the patch forward's decomposition, the tests of the new kernels (patch forward,
# fused densityopt, per-image colour transforms, mixed-fleet loader), the 1-rank RCCL step with and without the
# graph self-check stage, densityopt 70 epochs x 4 seeds on the fused iteration,
# its graph-only steady-state trace (launches and device copies per iteration) and the steady run's phases.
set -u
cd "$(dirname "$0")/../.."
O=gpurun_out/r6b2
mkdir -p $O
export TMPDIR=/tmp
trap 'find gpurun_out -type f -size +4M -print -delete; du -sh gpurun_out' EXIT
timeout -k 10 120 python -u -m pytest -q --timeout 100 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_conv_wgrad.py -k "decoded_patch" > $O/pytest_c4p.log 2>&1 || { tail -30 $O/pytest_c4p.log; exit 1; }
tail -2 $O/pytest_c4p.log
timeout -k 10 200 python scripts/c4w_bench.py --patch-only > $O/c4w_bench.jsonl 2>&1 || { tail -20 $O/c4w_bench.jsonl; exit 1; }
cat $O/c4w_bench.jsonl
for v in "c4p:" "c4w:BT_C4W_PATCH=0" "c4p:" "c4w:BT_C4W_PATCH=0"; do
  name=${v%%:*}; e=${v#*:}
  timeout -k 10 200 env $e BT_CONV_FWD_PATCH=0 python bench.py --consumer disc --steps 2000 > $O/disc.log 2>&1 || { tail -5 $O/disc.log; exit 1; }
  grep '^{' $O/disc.log | tee -a $O/disc_$name.jsonl | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'v':'$name','disc':d['value'],'ms':d['ms_per_step']}))"
done
timeout -k 10 120 python scripts/fwd_patch_bench.py > $O/fwd_patch_bench.jsonl 2>&1 || { tail -20 $O/fwd_patch_bench.jsonl; exit 1; }
cat $O/fwd_patch_bench.jsonl
timeout -k 10 400 python -u -m pytest -q --timeout 150 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_conv_wgrad.py tests/test_gpu_consumer.py tests/test_gpu_kernels.py tests/test_gpu_loader.py tests/test_adam.py \
  > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; grep -E "^(FAILED|ERROR)" $O/pytest.log | head -20
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for v in "graphcheck:" "nographcheck:BT_SELFCHECK_GRAPH=0"; do
  name=${v%%:*}; e=${v#*:}
  timeout -k 10 300 env $e python bench.py --consumer disc --force-pg --steps 1000 > $O/disc_pg1.log 2>&1 || { tail -20 $O/disc_pg1.log; exit 1; }
  grep '^{' $O/disc_pg1.log | tee -a $O/disc_pg1_$name.jsonl | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'v':'$name','pg1':d['value'],'sc':d['allreduce_check'].get('selfcheck')}))"
done
timeout -k 10 300 python examples/densityopt/densityopt.py --num-epochs 70 --num-runs 4 --image-every 0 \
  --out-dir $O/dopt_e70 --json $O/dopt_e70.json > $O/dopt_e70.log 2>&1 || { tail -5 $O/dopt_e70.log; exit 1; }
python -c "
import json; d=json.load(open('$O/dopt_e70.json'))
for r in d.get('runs',[d]): print(json.dumps({'it_s':round(r['iterations_per_s'],1),'steady':round(r['steady']['iterations_per_s'],1),'fused':r.get('fused_sstep'),'abs_diff':[round(x,3) for x in r['abs_diff']]}))"
timeout -k 10 240 rocprofv3 --kernel-trace -d /tmp/dtr_dopt -o run --output-format csv -- python examples/densityopt/densityopt.py --num-epochs 400 --image-every 0 --out-dir '' > $O/dopt_trace.log 2>&1 || { tail -5 $O/dopt_trace.log; exit 1; }
python scripts/dopt_iteration.py /tmp/dtr_dopt --iters 200 > $O/dopt_iteration_kernels.txt || exit 1
head -50 $O/dopt_iteration_kernels.txt
for v in "fused:" "unfused:--unfused-sstep"; do
  name=${v%%:*}; e=${v#*:}
  timeout -k 10 300 python examples/densityopt/densityopt.py --num-epochs 2000 --image-every 0 --out-dir '' $e \
    --json $O/dopt_steady_$name.json > $O/dopt_steady.log 2>&1 || { tail -5 $O/dopt_steady.log; exit 1; }
  python -c "import json; d=json.load(open('$O/dopt_steady_$name.json')); print(json.dumps({'v':'$name','it_s':round(d['iterations_per_s'],1),'steady':d['steady']['iterations_per_s'],'ms':d['steady']['ms_per_iteration'],'abs_diff':[round(x,3) for x in d['abs_diff']]}))"
done
BT_CONV_FWD_PATCH=0 bash scripts/gpurun/disc_trace.sh r6b2 > /dev/null || exit 1
cp gpurun_out/trace_r6b2/step_sequence.txt $O/disc_step_sequence_nopatch.txt
grep -A24 "mean over" $O/disc_step_sequence_nopatch.txt | head -30
