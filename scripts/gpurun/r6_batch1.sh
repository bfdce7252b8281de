#!/bin/bash
# Round 6, GPU session 1: the whole GPU suite (persistent patch forward for conv2, ordered slice reduce, grid-barrier flag, graph
# all-reduce self-check, determinism), smoke(), headline bench (2000 steps and a 20-step
# driver-like run with the sustained window), disc ordered vs atomic reduce, the disc step
# with a 1-rank RCCL group (self-check incl. the captured all-reduce stage), the 8-rank gloo
# rehearsal through bench.py's own supervisor, and a disc kernel trace.
set -u
cd "$(dirname "$0")/../.."
O=gpurun_out/r6b1
mkdir -p $O
export TMPDIR=/tmp
trap 'find gpurun_out -type f -size +4M -print -delete; du -sh gpurun_out' EXIT
timeout -k 10 900 python -u -m pytest -q --timeout 200 --timeout-method thread -p no:cacheprovider tests -m gpu \
  > $O/pytest_gpu.log 2>&1
rc=$?; tail -3 $O/pytest_gpu.log; grep -E "^(FAILED|ERROR)" $O/pytest_gpu.log | head -20
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python bench.py > $O/bench_default.log 2>&1 || { tail -5 $O/bench_default.log; exit 1; }
grep '^{' $O/bench_default.log | tee $O/bench_default.jsonl | cut -c1-300
timeout -k 10 300 python bench.py --steps 20 --warmup 10 > $O/bench_20.log 2>&1 || { tail -5 $O/bench_20.log; exit 1; }
grep '^{' $O/bench_20.log | tee $O/bench_20.jsonl | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'v20':d['value'],'backlog':d['backlog_covers_window'],'sustained':d['sustained']}))"
for v in "default:" "nopatch:BT_CONV_FWD_PATCH=0" "atomic:BT_WGRAD_ORDERED=0" "default:" "nopatch:BT_CONV_FWD_PATCH=0" "atomic:BT_WGRAD_ORDERED=0"; do
  name=${v%%:*}; e=${v#*:}
  timeout -k 10 200 env $e python bench.py --consumer disc --steps 2000 > $O/disc.log 2>&1 || { tail -5 $O/disc.log; exit 1; }
  grep '^{' $O/disc.log | tee -a $O/disc_$name.jsonl | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'v':'$name','disc':d['value'],'ms':d['ms_per_step']}))"
done
timeout -k 10 300 python bench.py --consumer disc --force-pg --steps 500 > $O/disc_pg1.log 2>&1 || { tail -20 $O/disc_pg1.log; exit 1; }
grep '^{' $O/disc_pg1.log | tee $O/disc_pg1.jsonl | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'pg1':d['value'],'check':d['allreduce_check'],'coll':d['config']['collectives'],'step':d['config']['consumer_step']}))"
