# kernel trace of the graphed discriminator step (microbench), per-kernel totals per step
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace -d /tmp/dkt -o run --output-format csv -- python scripts/disc_step_bench.py --only bf16-nhwc --graph on --iters 300 --cast fused --u8 --optim gfx950 --head fused > gpurun_out/dkt.log 2>&1 || { tail gpurun_out/dkt.log; exit 1; }
f=$(find /tmp/dkt -name '*kernel_trace.csv' | head -1)
python - "$f" <<'PY' > gpurun_out/disc_step_kernels.txt
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r['Start_Timestamp']))
rows = rows[-15000:]   # steady state
steps = 200
tot = collections.defaultdict(float); cnt = collections.Counter()
for r in rows:
    n = r['Kernel_Name']
    short = n.replace('(anonymous namespace)::', '').split('(')[0]
    short = short.replace('void ', '')[:90]
    tot[short] += (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1000
    cnt[short] += 1
span = (int(rows[-1]['End_Timestamp']) - int(rows[0]['Start_Timestamp'])) / 1000
busy = sum(tot.values())
print(f'last {len(rows)} kernels, span {span:.0f} us, busy {busy:.0f} us ({100*busy/span:.1f}%)')
ksteps = len(rows) / 1.0
for k, v in sorted(tot.items(), key=lambda kv: -kv[1])[:40]:
    print(f'{v:10.0f} us {cnt[k]:6d}x {v/cnt[k]:8.2f} us/call  {k}')
PY
head -45 gpurun_out/disc_step_kernels.txt
