#!/bin/bash
# Round 5, GPU session 8: fused data+weight gradient launch (A/B), the disc step's roofline data (trace + PMC passes:
# LDS bank conflicts, VALU/MFMA, HBM bytes) on the current kernels, the replay
# sampler's LDS counters, and the disc bench after the c4w revert.
set -u
cd "$(dirname "$0")/../.."
O=gpurun_out/r5b8
mkdir -p $O
export TMPDIR=/tmp
trap 'find gpurun_out -type f -size +4M -print -delete; du -sh gpurun_out' EXIT
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_conv_wgrad.py tests/test_gpu_consumer.py tests/test_replay.py -m gpu > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for v in "fused:" "twolaunch:BT_FUSE_DW=0" "fused:" "twolaunch:BT_FUSE_DW=0"; do
  name=${v%%:*}; e=${v#*:}
  timeout -k 10 200 env $e python bench.py --consumer disc --steps 2000 > $O/disc.log 2>&1 || { tail -5 $O/disc.log; exit 1; }
  grep '^{' $O/disc.log | tee -a $O/disc_$name.jsonl | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'v':'$name','disc':d['value'],'ms':d['ms_per_step']}))"
done
bash scripts/gpurun/disc_roofline.sh r5b8 > $O/roofline.log 2>&1 || { tail -20 $O/roofline.log; exit 1; }
cat gpurun_out/roof_r5b8/roofline.md
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --kernel-trace -d /tmp/rpmc_replay -o run --output-format csv -- python benchmarks/bench_replay.py --batch 64 --steps 100 --warmup 5 > $O/replay_pmc.log 2>&1 || { tail -5 $O/replay_pmc.log; exit 1; }
f=$(find /tmp/rpmc_replay -name '*counter_collection.csv' | head -1)
cp "$f" $O/replay_pmc.csv
python - <<'PY'
import csv, collections
rows = list(csv.DictReader(open('gpurun_out/r5b8/replay_pmc.csv')))
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for r in rows:
    k = r['Kernel_Name'][:60]
    agg[k][r['Counter_Name']] += float(r['Counter_Value'])
for k, v in agg.items():
    if v.get('SQ_LDS_IDX_ACTIVE'):
        print(k, {c: round(x) for c, x in v.items()}, 'conflict %', round(100 * v['SQ_LDS_BANK_CONFLICT'] / v['SQ_LDS_IDX_ACTIVE'], 1))
PY
for v in "uni:" "tbl:BT_REPLAY_UNI=0" "uni:" "tbl:BT_REPLAY_UNI=0"; do
  name=${v%%:*}; e=${v#*:}
  for b in 64 8; do
    timeout -k 10 120 env $e python benchmarks/bench_replay.py --batch $b --steps 2000 > $O/replay.log 2>&1 || { tail -5 $O/replay.log; exit 1; }
    grep '^{' $O/replay.log | tee -a $O/replay_${name}_b$b.jsonl | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'v':'$name','B':$b,'us':d['us_per_batch'],'tbps':d['effective_tbps']}))"
  done
done
# densityopt: the real-half prefetch against the inline iteration, same box, alternating
for v in "prefetch:" "inline:--no-prefetch" "prefetch:" "inline:--no-prefetch"; do
  name=${v%%:*}; flags=${v#*:}
  timeout -k 10 200 python examples/densityopt/densityopt.py --num-epochs 1000 --seed 0 --image-every 0 $flags \
    --out-dir '' --json $O/dopt_$name.json > $O/dopt.log 2>&1 || { tail -5 $O/dopt.log; exit 1; }
  python -c "
import json; d=json.load(open('$O/dopt_$name.json')); s=d['steady']; m=s['ms_per_iteration']
print(json.dumps({'v':'$name','it_s':round(s['iterations_per_s'],1),'wait_fetch_send_ms':round(m['sim_wait']+m['fetch']+m['send'],3),'ms':m,'abs_diff':[round(x,3) for x in d.get('abs_diff',[])]}))" | tee -a $O/dopt_ab.jsonl
done
