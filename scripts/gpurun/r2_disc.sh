set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_conv_wgrad.py tests/test_gpu_consumer.py tests/test_adam.py > gpurun_out/disc_tests.log 2>&1; rc=$?
tail -2 gpurun_out/disc_tests.log; [ $rc -eq 0 ] || { grep -B10 "Error\|assert" gpurun_out/disc_tests.log | head -60; exit $rc; }
run() { timeout -k 10 200 "$@" > gpurun_out/dp.log 2>&1 || { tail -5 gpurun_out/dp.log; exit 1; }; grep '^{' gpurun_out/dp.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$*'.replace('python bench.py',''), '->', d['value'], d['ms_per_step'], d.get('consumer_wait_ms_per_batch'), d.get('h2d_gbytes_per_s'))"; }
run python bench.py --consumer disc --steps 1000
run python bench.py --consumer disc --steps 3000
timeout -k 10 200 python scripts/disc_step_bench.py --only bf16-nhwc --graph on --iters 500 --cast fused --u8 --optim gfx950 --head fused | grep '^{'
