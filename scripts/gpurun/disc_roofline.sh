#!/bin/bash
# Roofline data for one disc consumer step: the graphed step's kernel trace
# (durations per position) and PMC passes over eager steps (counters per
# dispatch), combined by scripts/disc_roofline.py.  Usage: disc_roofline.sh TAG
set -u
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
tag=$1; shift
O=gpurun_out/roof_$tag
mkdir -p $O
bash scripts/gpurun/disc_trace.sh $tag "$@" > /dev/null || exit 1
cp gpurun_out/trace_$tag/step_sequence.txt $O/step_sequence.txt
rm -f gpurun_out/trace_$tag/bench.log
i=0
for ctr in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $ctr --kernel-trace -d /tmp/rpmc_$tag$i -o run --output-format csv -- python scripts/disc_step_bench.py --only bf16-nhwc --graph off --iters 4 --cast fused --u8 --optim gfx950 --head fused > $O/p$i.log 2>&1 || { tail -5 $O/p$i.log; exit 1; }
  f=$(find /tmp/rpmc_$tag$i -name '*counter_collection.csv' | head -1)
  cp "$f" $O/pass$i.csv
done
python scripts/disc_roofline.py $O/step_sequence.txt $O --md $O/roofline.md
