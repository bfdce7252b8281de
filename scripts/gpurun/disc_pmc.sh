#!/bin/bash
# PMC passes over the disc consumer step's kernels (eager steps, one dispatch each), summarised per kernel.
set -u
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
mkdir -p gpurun_out/disc_pmc
i=0
for ctr in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES" \
           "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE" \
           "FETCH_SIZE" "WRITE_SIZE TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $ctr --kernel-trace -d /tmp/dpmc$i -o run --output-format csv -- python scripts/disc_step_bench.py --only bf16-nhwc --graph off --iters 4 --cast fused --u8 --optim gfx950 --head fused > gpurun_out/disc_pmc/p$i.log 2>&1 || { tail -5 gpurun_out/disc_pmc/p$i.log; exit 1; }
  f=$(find /tmp/dpmc$i -name '*counter_collection.csv' | head -1)
  cp "$f" gpurun_out/disc_pmc/pass$i.csv
done
python - <<'PY' | tee gpurun_out/disc_pmc/summary.txt
import csv, glob, collections
agg = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(set)
for f in sorted(glob.glob('gpurun_out/disc_pmc/pass*.csv')):
    for r in csv.DictReader(open(f)):
        n = r['Kernel_Name'].replace('(anonymous namespace)::', '').replace('btn::gpu::', '').split('(')[0].replace('void ', '')[:60]
        agg[n][r['Counter_Name']] += float(r['Counter_Value'])
        disp[n].add(r['Dispatch_Id'])
print(f"{'kernel':60s} {'VALU/MFMA':>9s} {'LDS/MFMA':>8s} {'bankcf%':>7s} {'wait%':>6s} {'valu%':>6s} {'fetchMB':>8s} {'writeMB':>8s} {'L2hit%':>6s} {'waves':>7s}")
for n, d in sorted(agg.items(), key=lambda kv: -kv[1].get('SQ_WAVE_CYCLES', 0)):
    k = max(1, len(disp[n]) // 4)
    mf = d.get('SQ_INSTS_MFMA', 0)
    wc = d.get('SQ_WAVE_CYCLES', 0) or 1
    hit, miss = d.get('TCC_HIT_sum', 0), d.get('TCC_MISS_sum', 0)
    print(f"{n:60s} {d.get('SQ_INSTS_VALU',0)/mf if mf else 0:9.2f} {d.get('SQ_INSTS_LDS',0)/mf if mf else 0:8.2f} "
          f"{100*d.get('SQ_LDS_BANK_CONFLICT',0)/max(1,d.get('SQ_ACTIVE_INST_LDS',1)):7.1f} {100*d.get('SQ_WAIT_ANY',0)/wc:6.1f} "
          f"{100*d.get('SQ_ACTIVE_INST_VALU',0)/wc:6.1f} {2*d.get('FETCH_SIZE',0)/1024/k:8.1f} {d.get('WRITE_SIZE',0)/1024/k:8.1f} "
          f"{100*hit/max(1,hit+miss):6.1f} {d.get('SQ_WAVES',0)/k:7.0f}")
PY
