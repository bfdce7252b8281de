set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for q in 4 8 16; do
  for extra in "" "--h2d auto" "--consumer-input resident"; do
    GPU_MAX_HW_QUEUES=$q timeout -k 10 200 python bench.py --consumer disc --steps 500 $extra > gpurun_out/hwq.log 2>&1 || { echo "fail q=$q $extra"; tail -5 gpurun_out/hwq.log; exit 1; }
    grep '^{' gpurun_out/hwq.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('q=$q', '$extra', d['value'], d['ms_per_step'], d['consumer_wait_ms_per_batch'])"
  done
done
timeout -k 10 200 python scripts/disc_step_bench.py --only bf16-nhwc --graph on 2>&1 | grep '^{'
