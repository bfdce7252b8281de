# Bisect the consumer-step time between scripts/disc_step_bench.py (0.83 ms)
# and bench.py --consumer disc (~0.95 ms of kernels): weight-cast mode, u8
# input decoded inside the step, and MIOpen weight-gradient solver choice.
# Kernel stats of two variants land in gpurun_out/bisect_*.
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_adam.py tests/test_gpu_consumer.py > gpurun_out/adam_tests.log 2>&1; rc=$?; tail -15 gpurun_out/adam_tests.log; [ $rc -eq 0 ] || exit $rc
export TMPDIR=/tmp
mb() { timeout -k 10 200 env "$@" > gpurun_out/mb.log 2>&1; r=$?; grep "^{" gpurun_out/mb.log || { tail -20 gpurun_out/mb.log; exit 1; }; }
B="python scripts/disc_step_bench.py --only bf16-nhwc --graph on --iters 500"
mb $B --optim gfx950
mb $B
mb $B --cast fused
mb $B --u8
mb $B --cast fused --u8
mb MIOPEN_DEBUG_CONV_IMPLICIT_GEMM_ASM_WRW_GTC_XDLOPS_NHWC=0 $B --cast fused --u8
mb MIOPEN_DEBUG_CONV_IMPLICIT_GEMM_ASM_BWD_GTC_XDLOPS_NHWC=0 $B --cast fused --u8
mb MIOPEN_DEBUG_CONV_IMPLICIT_GEMM_ASM_FWD_GTC_XDLOPS_NHWC=0 $B --cast fused --u8
for v in "autocast" "fused --u8" "fused --u8 --optim gfx950"; do
  tag=$(echo $v | tr -d ' -')
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d /tmp/rp_$tag -o run --output-format csv -- \
    python scripts/disc_step_bench.py --only bf16-nhwc --graph on --iters 300 --cast $v > gpurun_out/bisect_$tag.log 2>&1 || exit 1
  f=$(find /tmp/rp_$tag -name '*kernel_stats.csv' | head -1)
  cp "$f" gpurun_out/bisect_${tag}_kernel_stats.csv
  python scripts/trace_timeline.py /tmp/rp_$tag --last 20000 > gpurun_out/bisect_${tag}_timeline.txt 2>&1
  head -30 gpurun_out/bisect_${tag}_timeline.txt
done
mb $B --cast fused --u8 --optim gfx950
