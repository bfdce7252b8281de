#!/bin/bash
# PMC passes over the conv kernels (scripts/conv_prof.py); summary to gpurun_out/conv_pmc/summary.txt
set -u
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out/conv_pmc
export TMPDIR=/tmp
trap 'find gpurun_out -type f -size +8M -delete' EXIT
i=0
for ctr in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD" \
           "SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MFMA SQ_INSTS_SALU GRBM_GUI_ACTIVE" \
           "FETCH_SIZE TCP_TCC_READ_REQ_sum"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $ctr -d /tmp/cpmc$i -o run --output-format csv -- python scripts/conv_prof.py --iters 3 > gpurun_out/conv_pmc/p$i.log 2>&1 || { tail -5 gpurun_out/conv_pmc/p$i.log; exit 1; }
  f=$(find /tmp/cpmc$i -name '*counter_collection.csv' | head -1)
  cp "$f" gpurun_out/conv_pmc/pass$i.csv
done
python - <<'PY' | tee gpurun_out/conv_pmc/summary.txt
import csv, glob, collections
agg = collections.defaultdict(lambda: collections.defaultdict(float))
meta = {}
for f in sorted(glob.glob('gpurun_out/conv_pmc/pass*.csv')):
    for r in csv.DictReader(open(f)):
        n = r['Kernel_Name']
        if 'conv_' not in n and 'tap_gemm' not in n: continue
        key = (n.split('(')[0][-45:], r.get('Grid_Size', '?'))
        agg[key][r['Counter_Name']] += float(r['Counter_Value'])
        meta[key] = (r.get('VGPR_Count', r.get('Arch_VGPR_Count', '?')), r.get('LDS_Block_Size', r.get('LDS_Size', '?')))
for k, v in agg.items():
    print(k, meta[k], {c: round(x / 3) for c, x in sorted(v.items())})
PY
