# PMC passes over the MFMA conv kernels (scripts/conv_prof.py, 3 iterations per shape)
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/conv_pmc
export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > gpurun_out/conv_pmc/counters.txt 2>&1 || true
i=0
for ctr in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_SALU" \
           "SQ_WAVE_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS TCC_HIT_sum TCC_MISS_sum" \
           "FETCH_SIZE GRBM_GUI_ACTIVE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $ctr -d /tmp/cpmc$i -o run --output-format csv -- python scripts/conv_prof.py --iters 3 > gpurun_out/conv_pmc/p$i.log 2>&1 || { tail -5 gpurun_out/conv_pmc/p$i.log; exit 1; }
  f=$(find /tmp/cpmc$i -name '*counter_collection.csv' | head -1)
  cp "$f" gpurun_out/conv_pmc/pass$i.csv
done
python - <<'PY'
import csv, glob, collections
agg = collections.defaultdict(lambda: collections.defaultdict(float))
meta = {}
for f in sorted(glob.glob('gpurun_out/conv_pmc/pass*.csv')):
    for r in csv.DictReader(open(f)):
        n = r['Kernel_Name']
        if 'conv_' not in n and 'tap_gemm' not in n: continue
        key = (n.split('(')[0][-48:], r.get('Grid_Size', '?'))
        agg[key][r['Counter_Name']] += float(r['Counter_Value'])
        meta[key] = (r.get('VGPR_Count', r.get('Arch_VGPR_Count', '?')), r.get('LDS_Block_Size', r.get('LDS_Size', '?')))
for k, v in agg.items():
    d = {c: x / 3 for c, x in v.items()}
    w = max(d.get('SQ_WAVES', 1), 1)
    mf = d.get('SQ_INSTS_MFMA', 0)
    extra = {}
    if mf:
        extra['VALU/MFMA'] = round(d.get('SQ_INSTS_VALU', 0) / mf, 2)
        extra['LDS/MFMA'] = round(d.get('SQ_INSTS_LDS', 0) / mf, 2)
    if d.get('SQ_WAVE_CYCLES'):
        extra['wait_any/wave_cyc'] = round(d.get('SQ_WAIT_INST_ANY', 0) / d['SQ_WAVE_CYCLES'], 3)
        extra['wait_lds/wave_cyc'] = round(d.get('SQ_WAIT_INST_LDS', 0) / d['SQ_WAVE_CYCLES'], 3)
    print(k, meta[k], {c: round(x) for c, x in sorted(d.items())}, extra)
PY
