# where does the streamed consumer step lose time? (profiles/r2/disc_probe.txt)
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for load in 0 8 14; do
  timeout -k 10 200 python scripts/disc_step_bench.py --only bf16-nhwc --graph on --iters 500 --cpu-load $load 2>&1 | grep '^{' || exit 1
done
run() { timeout -k 10 200 env "$@" > gpurun_out/dp.log 2>&1 || { tail -5 gpurun_out/dp.log; exit 1; }; grep '^{' gpurun_out/dp.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$*'.replace('python bench.py',''), '->', d['value'], d['ms_per_step'], d['consumer_wait_ms_per_batch'], d['config'].get('cast'))"; }
run python bench.py --consumer disc --steps 1000
run python bench.py --consumer disc --steps 1000 --cast autocast
run BT_CUDNN_BENCHMARK=0 python bench.py --consumer disc --steps 1000
run python bench.py --consumer disc --steps 1000 --producers 2
run python bench.py --consumer disc --steps 1000 --producers 4
run python bench.py --consumer disc --steps 1000 --producers 2 --consumer-input resident
