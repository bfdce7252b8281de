#!/bin/bash
# Round 5, GPU session 1: densityopt over 2000 epochs in both formulations
# (bf16 graphed default vs fp32 eager, same seed), and config 5 (cart-pole
# RemoteEnv, 8 and 32 envs) re-measured on the current transport.
set -u
cd "$(dirname "$0")/../.."
O=gpurun_out/r5b1
mkdir -p $O
export TMPDIR=/tmp
trap 'find gpurun_out -type f -size +4M -print -delete; du -sh gpurun_out' EXIT
for v in "bf16graph:" "fp32eager:--fp32 --no-graph"; do
  name=${v%%:*}; flags=${v#*:}
  timeout -k 10 400 python examples/densityopt/densityopt.py --num-epochs 2000 --seed 0 --image-every 0 $flags \
    --out-dir $O/dopt_$name --json $O/dopt_$name.json > $O/dopt_$name.log 2>&1 || { tail -5 $O/dopt_$name.log; exit 1; }
  python -c "import json; d=json.load(open('$O/dopt_$name.json')); print('$name', json.dumps({k: d.get(k) for k in ('iterations_per_s','abs_diff','final_params','steady')})[:600])"
done
for e in 8 32; do
  timeout -k 10 300 python benchmarks/bench_rl.py --envs $e --steps 5000 > $O/rl_$e.log 2>&1 || { tail -5 $O/rl_$e.log; exit 1; }
  grep '^{' $O/rl_$e.log | tee -a $O/rl.jsonl | cut -c1-300
done
# fair fan-in: the headline with 5 (uneven over 4 IO sockets) and 8 producers
for p in 5 8; do
  timeout -k 10 300 python bench.py --producers $p --steps 2000 > $O/headline_p$p.log 2>&1 || { tail -5 $O/headline_p$p.log; exit 1; }
  grep '^{' $O/headline_p$p.log | tee -a $O/headline.jsonl | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'p':$p,'value':d['value'],'share':d['producer_share_max_over_min'],'per':d['producer_frames_per_s'],'backlog':d['backlog_covers_window']}))"
done
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_loader.py tests/test_gpu_consumer.py -m gpu > $O/pytest_loader_consumer.log 2>&1
rc=$?; tail -3 $O/pytest_loader_consumer.log; grep -E "^(FAILED|ERROR)" $O/pytest_loader_consumer.log | head; exit $rc
