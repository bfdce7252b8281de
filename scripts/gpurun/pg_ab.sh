#!/bin/bash
# Why does a 1-rank RCCL process group slow scatter mode?  Same box, 2000 steps each.
set -u
cd "$(dirname "$0")/../.."
a="--dist scatter --steps 2000 --prefetch 12"
run() { echo "== $1"; shift; timeout -k 10 200 env "$@" python bench.py $a --force-pg > gpurun_out/pgab.log 2>&1 || { tail -5 gpurun_out/pgab.log; return 1; }
        grep '^{' gpurun_out/pgab.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])"; }
timeout -k 10 200 python bench.py $a > gpurun_out/pgab.log 2>&1 && grep '^{' gpurun_out/pgab.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('no pg', d['value'])"
run "pg default" X=1
run "pg no DeviceComm" BT_NO_DEVICECOMM=1
run "pg no monitoring/async errors" TORCH_NCCL_ENABLE_MONITORING=0 TORCH_NCCL_ASYNC_ERROR_HANDLING=0 TORCH_NCCL_DUMP_ON_TIMEOUT=0
run "pg no DeviceComm + no monitoring" BT_NO_DEVICECOMM=1 TORCH_NCCL_ENABLE_MONITORING=0 TORCH_NCCL_ASYNC_ERROR_HANDLING=0 TORCH_NCCL_DUMP_ON_TIMEOUT=0
