#!/bin/bash
# conv kernel iteration: numerics, per-layer timings, disc consumer bench
set -u
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
export TMPDIR=/tmp
trap 'find gpurun_out -type f -size +8M -delete' EXIT
timeout -k 10 240 python -c "import sys; sys.path.insert(0,'.'); import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || { tail -20 gpurun_out/build.log; exit 2; }
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_conv_wgrad.py tests/test_gpu_kernels.py tests/test_gpu_consumer.py > gpurun_out/conv_tests.log 2>&1; rc=$?
tail -3 gpurun_out/conv_tests.log; [ $rc -eq 0 ] || { grep -B5 Error gpurun_out/conv_tests.log | head -40; exit $rc; }
timeout -k 10 200 python scripts/conv_bench.py > gpurun_out/conv_bench.log 2>&1; rc=$?; grep '^{' gpurun_out/conv_bench.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python scripts/disc_step_bench.py --only bf16-nhwc --graph on --cast fused --optim gfx950 --head fused --u8 --iters 1000 > gpurun_out/dstep_res.log 2>&1; rc=$?; grep '^{' gpurun_out/dstep_res.log | cut -c1-400; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --consumer disc --steps 300 > gpurun_out/disc.log 2>&1; rc=$?; grep '^{' gpurun_out/disc.log | cut -c1-200; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/rp_ktd -o run --output-format csv -- python bench.py --consumer disc --steps 300 > gpurun_out/ktd.log 2>&1; rc=$?
python scripts/trace_timeline.py /tmp/rp_ktd --last 13000 > gpurun_out/ktd.txt 2>&1; head -32 gpurun_out/ktd.txt
exit $rc
