#!/bin/bash
# Round 6, GPU session 1b: the 8-rank gloo rehearsal through bench.py's own supervisor, the
# mixed shm + inline fleet against an all-shm fleet, the TCP inline path (4 and 8 producers,
# one IO thread per pipe vs the old cap of 4), and a disc kernel trace.
set -u
cd "$(dirname "$0")/../.."
O=gpurun_out/r6b1
mkdir -p $O
export TMPDIR=/tmp
trap 'find gpurun_out -type f -size +4M -print -delete; du -sh gpurun_out' EXIT
summ() { python -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'v':'$1','img_s':d['value'],'share':d.get('producer_share_max_over_min'),'direct':d['loader_stats'].get('direct_batches'),'batches':d['loader_stats'].get('batches'),'staged':d['loader_stats'].get('staged_frames'),'fallbacks':d['loader_stats'].get('pool_fallbacks'),'cpu':d.get('cpu',{}).get('us_per_frame')}))"; }
for v in "jitter:--color-jitter" "shm6:--producers 6" "mixed3x3:--producers 6 --inline-producers 3" "tcp4:--proto tcp --shm 0 --producers 4" "tcp4_io4:--proto tcp --shm 0 --producers 4 --io-threads 4" "tcp8:--proto tcp --shm 0 --producers 8" "tcp8_io4:--proto tcp --shm 0 --producers 8 --io-threads 4" "ipc8_inline:--shm 0 --producers 8"; do
  name=${v%%:*}; a=${v#*:}
  timeout -k 10 240 python bench.py $a --steps 2000 > $O/fleet.log 2>&1 || { tail -5 $O/fleet.log; exit 1; }
  grep '^{' $O/fleet.log | tee -a $O/fleet_$name.jsonl | summ $name
done
timeout -k 10 400 python bench.py --gpus 8 --backend gloo --steps 300 --warmup 30 > $O/gloo8.log 2>&1 || { tail -30 $O/gloo8.log; exit 1; }
grep '^{' $O/gloo8.log | tee $O/gloo8.jsonl | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'gloo8':d['value'],'seen':d['world_size_seen'],'rates':[r['images_per_s'] for r in d['per_rank']],'prod':[r['producers'] for r in d['per_rank']],'cpus':[r['cpus'] for r in d['per_rank']]}))"
bash scripts/gpurun/disc_trace.sh r6b1 > /dev/null || exit 1
cp gpurun_out/trace_r6b1/step_sequence.txt $O/disc_step_sequence.txt
grep -A22 "mean over" $O/disc_step_sequence.txt
grep "busy\|median step" $O/disc_step_sequence.txt
