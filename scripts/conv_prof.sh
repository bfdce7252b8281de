set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for b in 256 1024; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d /tmp/cp$b -o run --output-format csv -- python scripts/conv_prof.py --blocks $b > gpurun_out/cp.log 2>&1 || { tail gpurun_out/cp.log; exit 1; }
  f=$(find /tmp/cp$b -name '*kernel_trace.csv' | head -1)
  python - "$f" $b <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
d = collections.defaultdict(list)
for r in rows:
    n = r['Kernel_Name']
    if 'conv_' not in n: continue
    key = n.split('(')[0].split('::')[-1] + ' grid=' + r.get('Grid_Size', r.get('Grid_Size_X', '?'))
    d[key].append((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1000)
for k, v in sorted(d.items()):
    v = sorted(v)
    print(f"blocks={sys.argv[2]} {k:70s} n={len(v):4d} median={v[len(v)//2]:8.2f} us")
PY
done
