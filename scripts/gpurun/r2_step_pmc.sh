#!/bin/bash
# PMC passes over the discriminator training step (eager, resident batch, bench config): per-kernel
# MFMA / VALU / LDS instruction counts, bank conflicts, busy cycles and HBM bytes -> gpurun_out/step_pmc/summary.txt
set -u
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out/step_pmc
export TMPDIR=/tmp
trap 'find gpurun_out -type f -size +8M -delete' EXIT
CMD="python scripts/disc_step_bench.py --only bf16-nhwc --graph off --cast fused --optim gfx950 --head fused --u8 --iters 4"
i=0
for ctr in "SQ_WAVES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD" \
           "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $ctr --kernel-trace -d /tmp/spmc$i -o run --output-format csv -- $CMD > gpurun_out/step_pmc/p$i.log 2>&1 || { tail -5 gpurun_out/step_pmc/p$i.log; exit 1; }
  f=$(find /tmp/spmc$i -name '*counter_collection.csv' | head -1)
  cp "$f" gpurun_out/step_pmc/pass$i.csv
done
python - <<'PY' | tee gpurun_out/step_pmc/summary.txt
import csv, glob, collections
agg = collections.defaultdict(lambda: collections.defaultdict(float))
calls = collections.defaultdict(set)
for f in sorted(glob.glob('gpurun_out/step_pmc/pass*.csv')):
    for r in csv.DictReader(open(f)):
        n = r['Kernel_Name'].split('(')[0].replace('btn::gpu::', '').replace('(anonymous namespace)::', '').replace('void ', '')[:48]
        agg[n][r['Counter_Name']] += float(r['Counter_Value'])
        calls[(n, r['Counter_Name'])].add(r.get('Dispatch_Id', r.get('Correlation_Id', len(calls))))
print(f"{'kernel':48s} {'calls':>5s} {'MFMA/wave':>9s} {'VALU/MFMA':>9s} {'LDSconf/LDS':>11s} {'MFMAbusy%':>9s} {'FETCH MB':>9s} {'WRITE MB':>9s}")
for n, v in sorted(agg.items(), key=lambda kv: -kv[1].get('SQ_INSTS_MFMA', 0)):
    k = max(1, len(calls[(n, 'SQ_WAVES')]))
    mf = v.get('SQ_INSTS_MFMA', 0)
    waves = v.get('SQ_WAVES', 1) or 1
    busy = v.get('SQ_VALU_MFMA_BUSY_CYCLES', 0) / max(1.0, v.get('GRBM_GUI_ACTIVE', 0)) * 100
    print(f"{n:48s} {k:5d} {mf / waves:9.1f} {v.get('SQ_INSTS_VALU', 0) / max(1, mf):9.2f} "
          f"{v.get('SQ_LDS_BANK_CONFLICT', 0) / max(1, v.get('SQ_INSTS_LDS', 0)):11.2f} {busy:9.1f} "
          f"{v.get('FETCH_SIZE', 0) / k / 1024:9.1f} {v.get('WRITE_SIZE', 0) / k / 1024:9.1f}")
PY
