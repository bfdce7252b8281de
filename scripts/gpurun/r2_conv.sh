# GPU tests of the round-2 consumer ops, then the wgrad kernel timing and the DMA-phase probe
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -s -m gpu tests/test_conv_wgrad.py tests/test_adam.py tests/test_gpu_consumer.py tests/test_gpu_loader.py > gpurun_out/r2_tests.log 2>&1; rc=$?
tail -25 gpurun_out/r2_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python scripts/conv_bench.py > gpurun_out/conv_bench.log 2>&1; rc=$?; cat gpurun_out/conv_bench.log | tail -5; [ $rc -eq 0 ] || exit $rc
bash scripts/dma_phase.sh
run() { timeout -k 10 200 "$@" > gpurun_out/dp.log 2>&1 || { tail -5 gpurun_out/dp.log; exit 1; }; grep '^{' gpurun_out/dp.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$*'.replace('python bench.py',''), '->', d['value'], d['ms_per_step'], d['consumer_wait_ms_per_batch'], d['config'].get('dma_phase'))"; }
run python bench.py --consumer disc --steps 1000
run python bench.py --consumer disc --steps 1000 --dma-phase mid
run python bench.py --consumer disc --steps 1000 --dma-phase mid --copy-streams 1
