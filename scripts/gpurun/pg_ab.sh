#!/bin/bash
# Why does a 1-rank RCCL process group slow scatter mode?  Same box, 2000 steps each,
# with the busiest threads of the consumer process over the timed region.
set -u
cd "$(dirname "$0")/../.."
a="--dist scatter --steps 2000 --prefetch 12"
show() { grep '^{' gpurun_out/pgab.log | python -c "
import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d.get('cpu', {}).get('threads_cpu_s'), d.get('cpu', {}).get('consumer_cpu_s'))"; }
run() { echo "== $1"; shift; timeout -k 10 200 env BT_THREAD_REPORT=1 "$@" python bench.py $a --force-pg > gpurun_out/pgab.log 2>&1 || { tail -5 gpurun_out/pgab.log; return 1; }; show; }
echo "== no pg"
timeout -k 10 200 env BT_THREAD_REPORT=1 python bench.py $a > gpurun_out/pgab.log 2>&1 && show
run "pg default (shared DeviceComm)" X=1
run "pg no DeviceComm" BT_NO_DEVICECOMM=1
run "pg dedicated DeviceComm" BT_DEVICECOMM_DEDICATED=1
