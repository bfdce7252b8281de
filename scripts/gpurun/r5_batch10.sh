#!/bin/bash
# Round 5, GPU session 10: the Adam schedule riding in the backward's last
# slice-reduce launch (A/B against its own launch) and the step trace.
set -u
cd "$(dirname "$0")/../.."
O=gpurun_out/r5b10
mkdir -p $O
export TMPDIR=/tmp
trap 'find gpurun_out -type f -size +4M -print -delete; du -sh gpurun_out' EXIT
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_adam.py tests/test_gpu_consumer.py tests/test_conv_wgrad.py -m gpu > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 env BT_C4W_LDS_COEF=1 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_conv_wgrad.py -m gpu -k "first or c4 or rgba or bn_backward or side or fused" > $O/pytest_ldsc.log 2>&1 || { tail -30 $O/pytest_ldsc.log; exit 1; }
tail -2 $O/pytest_ldsc.log
timeout -k 10 300 env BT_C4W_LDS_COEF=1 python scripts/c4w_bench.py --iters 200 > $O/c4w_bench_ldsc.jsonl 2>&1 || { tail -5 $O/c4w_bench_ldsc.jsonl; exit 1; }
timeout -k 10 300 python scripts/c4w_bench.py --iters 200 > $O/c4w_bench.jsonl 2>&1 || { tail -5 $O/c4w_bench.jsonl; exit 1; }
grep '"bn_dy": true, "u8": true, "waves": 4' $O/c4w_bench_ldsc.jsonl | sed 's/^/ldsc /'
grep '"bn_dy": true, "u8": true, "waves": 4' $O/c4w_bench.jsonl | sed 's/^/base /'
for v in "attach:" "own:BT_ADAM_ATTACH=0" "ldsc768:BT_C4W_LDS_COEF=1 BT_C4W_BLOCKS=768" "ldsc512:BT_C4W_LDS_COEF=1" "w8:BT_C4W_WAVES=8 BT_C4W_BLOCKS=256" "attach:" "own:BT_ADAM_ATTACH=0" "ldsc768:BT_C4W_LDS_COEF=1 BT_C4W_BLOCKS=768" "ldsc512:BT_C4W_LDS_COEF=1" "w8:BT_C4W_WAVES=8 BT_C4W_BLOCKS=256"; do
  name=${v%%:*}; e=${v#*:}
  timeout -k 10 200 env $e python bench.py --consumer disc --steps 2000 > $O/disc.log 2>&1 || { tail -5 $O/disc.log; exit 1; }
  grep '^{' $O/disc.log | tee -a $O/disc_$name.jsonl | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'v':'$name','disc':d['value'],'ms':d['ms_per_step']}))"
done
bash scripts/gpurun/disc_trace.sh r5b10 > /dev/null || exit 1
cp gpurun_out/trace_r5b10/step_sequence.txt $O/disc_step_sequence.txt
grep -A21 "mean over" $O/disc_step_sequence.txt
grep "busy\|median step" $O/disc_step_sequence.txt
