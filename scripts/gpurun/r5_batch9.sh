#!/bin/bash
# Round 5, GPU session 9: the conflict-free replay table with 4 groups in
# flight per lane on a 4-block-per-CU grid (BT_REPLAY_UNI=1) against the
# per-channel table; the patch data gradient's shared launch (BT_FUSE_PATCH).
set -u
cd "$(dirname "$0")/../.."
O=gpurun_out/r5b9
mkdir -p $O
export TMPDIR=/tmp
trap 'find gpurun_out -type f -size +4M -print -delete; du -sh gpurun_out' EXIT
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_replay.py tests/test_gpu_kernels.py -m gpu > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 env BT_REPLAY_UNI=1 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_replay.py -m gpu > $O/pytest_uni.log 2>&1 || { tail -30 $O/pytest_uni.log; exit 1; }
tail -2 $O/pytest_uni.log
for v in "uni:BT_REPLAY_UNI=1" "tbl:" "uni:BT_REPLAY_UNI=1" "tbl:" "uni512:BT_REPLAY_UNI=1 BT_REPLAY_UNI_GRID=512" "uni2048:BT_REPLAY_UNI=1 BT_REPLAY_UNI_GRID=2048"; do
  name=${v%%:*}; e=${v#*:}
  for b in 64 8; do
    timeout -k 10 120 env $e python benchmarks/bench_replay.py --batch $b --steps 2000 > $O/replay.log 2>&1 || { tail -5 $O/replay.log; exit 1; }
    grep '^{' $O/replay.log | tee -a $O/replay_${name}_b$b.jsonl | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'v':'$name','B':$b,'us':d['us_per_batch'],'tbps':d['effective_tbps']}))"
  done
done
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --kernel-trace -d /tmp/rpmc_replay9 -o run --output-format csv -- python benchmarks/bench_replay.py --batch 64 --steps 100 --warmup 5 > $O/replay_pmc_tbl.log 2>&1 || { tail -5 $O/replay_pmc_tbl.log; exit 1; }
f=$(find /tmp/rpmc_replay9 -name '*counter_collection.csv' | head -1)
cp "$f" $O/replay_pmc_tbl.csv
for v in "patch:" "nopatch:BT_FUSE_PATCH=0" "patch:" "nopatch:BT_FUSE_PATCH=0"; do
  name=${v%%:*}; e=${v#*:}
  timeout -k 10 200 env $e python bench.py --consumer disc --steps 2000 > $O/disc.log 2>&1 || { tail -5 $O/disc.log; exit 1; }
  grep '^{' $O/disc.log | tee -a $O/disc_$name.jsonl | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'v':'$name','disc':d['value'],'ms':d['ms_per_step']}))"
done
