#!/bin/bash
# Round 6, GPU session 4: the decoded-patch first-layer weight gradient with a 4-deep dY ring,
# 128-channel weight-gradient tiles by default, densityopt's second gradient contributions added
# in the Adam kernel (no AccumulateGrad launches), then the loader fleet measurements: colour
# jitter, mixed shm + inline producers, TCP with one IO thread per pipe.
set -u
cd "$(dirname "$0")/../.."
O=gpurun_out/r6b4
mkdir -p $O
export TMPDIR=/tmp
trap 'find gpurun_out -type f -size +4M -print -delete; du -sh gpurun_out' EXIT
timeout -k 10 400 python -u -m pytest -q --timeout 150 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_conv_wgrad.py tests/test_gpu_consumer.py tests/test_adam.py tests/test_densityopt.py > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; grep -E "^(FAILED|ERROR)" $O/pytest.log | head -20
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 200 python scripts/c4w_bench.py --patch-only > $O/c4w_bench.jsonl 2>&1 || { tail -20 $O/c4w_bench.jsonl; exit 1; }
timeout -k 10 200 python scripts/wgrad_tiles_bench.py > $O/wgrad_tiles.jsonl 2>&1 || { tail -20 $O/wgrad_tiles.jsonl; exit 1; }
cat $O/wgrad_tiles.jsonl
cat $O/c4w_bench.jsonl
for v in "default:" "default:"; do
  name=${v%%:*}; e=${v#*:}
  timeout -k 10 200 env $e python bench.py --consumer disc --steps 2000 > $O/disc.log 2>&1 || { tail -5 $O/disc.log; exit 1; }
  grep '^{' $O/disc.log | tee -a $O/disc_$name.jsonl | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'v':'$name','disc':d['value'],'ms':d['ms_per_step']}))"
done
timeout -k 10 300 python examples/densityopt/densityopt.py --num-epochs 2000 --image-every 0 --out-dir '' \
  --json $O/dopt_steady.json > $O/dopt_steady.log 2>&1 || { tail -5 $O/dopt_steady.log; exit 1; }
python -c "import json; d=json.load(open('$O/dopt_steady.json')); print(json.dumps({'it_s':round(d['iterations_per_s'],1),'steady':d['steady']['iterations_per_s'],'ms':d['steady']['ms_per_iteration']}))"
timeout -k 10 240 rocprofv3 --kernel-trace -d /tmp/dtr_dopt -o run --output-format csv -- python examples/densityopt/densityopt.py --num-epochs 400 --image-every 0 --out-dir '' > $O/dopt_trace.log 2>&1 || { tail -5 $O/dopt_trace.log; exit 1; }
python scripts/dopt_iteration.py /tmp/dtr_dopt --iters 200 > $O/dopt_iteration_kernels.txt || exit 1
head -30 $O/dopt_iteration_kernels.txt
summ() { python -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'v':'$1','img_s':d['value'],'share':d.get('producer_share_max_over_min'),'direct':d['loader_stats'].get('direct_batches'),'batches':d['loader_stats'].get('batches'),'staged':d['loader_stats'].get('staged_frames'),'fallbacks':d['loader_stats'].get('pool_fallbacks'),'cpu':d.get('cpu',{}).get('us_per_frame')}))"; }
for v in "jitter:--color-jitter" "shm6:--producers 6" "mixed3x3:--producers 6 --inline-producers 3" "tcp4:--proto tcp --shm 0 --producers 4" "tcp4_io4:--proto tcp --shm 0 --producers 4 --io-threads 4" "tcp8:--proto tcp --shm 0 --producers 8" "tcp8_io4:--proto tcp --shm 0 --producers 8 --io-threads 4"; do
  name=${v%%:*}; a=${v#*:}
  timeout -k 10 240 python bench.py $a --steps 2000 > $O/fleet.log 2>&1 || { tail -5 $O/fleet.log; exit 1; }
  grep '^{' $O/fleet.log | tee -a $O/fleet_$name.jsonl | summ $name
done
