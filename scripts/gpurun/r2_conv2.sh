set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_conv_wgrad.py > gpurun_out/conv_tests.log 2>&1; rc=$?
tail -3 gpurun_out/conv_tests.log; [ $rc -eq 0 ] || { grep -B5 Error gpurun_out/conv_tests.log | head -40; exit $rc; }
timeout -k 10 200 python scripts/conv_bench.py > gpurun_out/conv_bench.log 2>&1; rc=$?; cat gpurun_out/conv_bench.log | grep '^{'; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python scripts/hip_api_cost.py
