#!/bin/bash
# Streaming vs a live process group, every variant in ONE call (same box).
# Usage: pg_tax.sh [steps]
set -u
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
S=${1:-2000}
run() {   # tag, env assignment (or X=0), bench args...
  local tag=$1 e=$2; shift 2
  timeout -k 10 200 env $e python bench.py --steps $S "$@" > gpurun_out/pg_$tag.log 2>&1 || { echo "FAIL $tag"; tail -5 gpurun_out/pg_$tag.log; return 1; }
  grep '^{' gpurun_out/pg_$tag.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'tag':'$tag','value':d['value'],'ms':d['ms_per_step'],'pg':d.get('pg_backend'),'sc':(d.get('allreduce_check') or {}).get('selfcheck'),'cpu':d['cpu']}))" | tee -a gpurun_out/pg_tax.jsonl
}
for mode in shard scatter; do
  run ${mode}_nopg X=0 --dist $mode && \
  run ${mode}_pg_nccl X=0 --dist $mode --force-pg --pg-backend nccl && \
  run ${mode}_pg_auto X=0 --dist $mode --force-pg && \
  run ${mode}_nopg_q8 GPU_MAX_HW_QUEUES=8 --dist $mode && \
  run ${mode}_pg_nccl_q8 GPU_MAX_HW_QUEUES=8 --dist $mode --force-pg --pg-backend nccl || exit 1
done
run shard_nopg_again X=0 --dist shard
