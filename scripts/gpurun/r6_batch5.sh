#!/bin/bash
# Round 6, GPU session 5: densityopt with fresh bucket views in its fused path (second gradient
# contributions added by the Adam kernel), the c4p ring back at depth 2, 128-channel data-gradient
# tiles in the fused pair and 256-column weight-gradient tiles fused with the patch data gradient
# (A/B), the 8-rank gloo rehearsal through bench.py's own supervisor, and the disc step trace.
set -u
cd "$(dirname "$0")/../.."
O=gpurun_out/r6b5
mkdir -p $O
export TMPDIR=/tmp
trap 'find gpurun_out -type f -size +4M -print -delete; du -sh gpurun_out' EXIT
timeout -k 10 400 python -u -m pytest -q --timeout 150 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_conv_wgrad.py tests/test_gpu_consumer.py tests/test_densityopt.py > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; grep -E "^(FAILED|ERROR)" $O/pytest.log | head -20
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 200 python scripts/wgrad_tiles_bench.py > $O/wgrad_tiles.jsonl 2>&1 || { tail -20 $O/wgrad_tiles.jsonl; exit 1; }
cat $O/wgrad_tiles.jsonl
timeout -k 10 200 python scripts/c4w_bench.py --patch-only > $O/c4w_bench.jsonl 2>&1 || { tail -20 $O/c4w_bench.jsonl; exit 1; }
cat $O/c4w_bench.jsonl
for v in "default:" "dbn128:BT_DGRAD_BN128=1" "wide:BT_WGRAD_WIDE=1" "red1:BT_REDUCE_ROUNDS=1" "bn128all:BT_CONV_BN=128" "default:" "dbn128:BT_DGRAD_BN128=1" "wide:BT_WGRAD_WIDE=1" "red1:BT_REDUCE_ROUNDS=1" "bn128all:BT_CONV_BN=128"; do
  name=${v%%:*}; e=${v#*:}
  timeout -k 10 200 env $e python bench.py --consumer disc --steps 2000 > $O/disc.log 2>&1 || { tail -5 $O/disc.log; exit 1; }
  grep '^{' $O/disc.log | tee -a $O/disc_$name.jsonl | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'v':'$name','disc':d['value'],'ms':d['ms_per_step']}))"
done
timeout -k 10 300 python examples/densityopt/densityopt.py --num-epochs 2000 --image-every 0 --out-dir '' \
  --json $O/dopt_steady.json > $O/dopt_steady.log 2>&1 || { tail -5 $O/dopt_steady.log; exit 1; }
python -c "import json; d=json.load(open('$O/dopt_steady.json')); print(json.dumps({'it_s':round(d['iterations_per_s'],1),'steady':d['steady']['iterations_per_s'],'ms':d['steady']['ms_per_iteration']}))"
timeout -k 10 300 python examples/densityopt/densityopt.py --num-epochs 70 --num-runs 4 --image-every 0 \
  --out-dir $O/dopt_e70 --json $O/dopt_e70.json > $O/dopt_e70.log 2>&1 || { tail -5 $O/dopt_e70.log; exit 1; }
python -c "
import json; d=json.load(open('$O/dopt_e70.json'))
for r in d.get('runs',[d]): print(json.dumps({'it_s':round(r['iterations_per_s'],1),'abs_diff':[round(x,3) for x in r['abs_diff']]}))"
timeout -k 10 240 rocprofv3 --kernel-trace -d /tmp/dtr_dopt -o run --output-format csv -- python examples/densityopt/densityopt.py --num-epochs 400 --image-every 0 --out-dir '' > $O/dopt_trace.log 2>&1 || { tail -5 $O/dopt_trace.log; exit 1; }
python scripts/dopt_iteration.py /tmp/dtr_dopt --iters 200 > $O/dopt_iteration_kernels.txt || exit 1
head -30 $O/dopt_iteration_kernels.txt
timeout -k 10 400 python bench.py --gpus 8 --backend gloo --steps 300 --warmup 30 > $O/gloo8.log 2>&1 || { tail -30 $O/gloo8.log; exit 1; }
grep '^{' $O/gloo8.log | tee $O/gloo8.jsonl | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'gloo8':d['value'],'seen':d['world_size_seen'],'rates':[r['images_per_s'] for r in d['per_rank']],'prod':[r['producers'] for r in d['per_rank']],'cpus':[r['cpus'] for r in d['per_rank']]}))"
bash scripts/gpurun/disc_trace.sh r6b5 > /dev/null || exit 1
cp gpurun_out/trace_r6b5/step_sequence.txt $O/disc_step_sequence.txt
grep -A24 "mean over" $O/disc_step_sequence.txt | head -30
