#!/bin/bash
# Decode value-transform A/B (scripts/decode_ab.py): timings for three
# variants, then LDS-conflict PMC passes for each.  Writes gpurun_out/decode_ab/.
set -u
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
out=gpurun_out/decode_ab
mkdir -p $out
timeout -k 10 240 python -c "import sys; sys.path.insert(0,'.'); import __graft_entry__ as g; g.build()" > $out/build.log 2>&1 || exit 2
for v in "0 32" "1 32" "1 16"; do
  set -- $v
  BLENDTORCH_DECODE_XFORM=$1 BLENDTORCH_GAMMA_COPIES=$2 timeout -k 10 120 python scripts/decode_ab.py >> $out/timing.jsonl 2> $out/timing_$1_$2.err || exit $?
done
for v in "0 32" "1 32" "1 16"; do
  set -- $v
  BLENDTORCH_DECODE_XFORM=$1 BLENDTORCH_GAMMA_COPIES=$2 timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_WAVES SQ_BUSY_CYCLES --kernel-trace -d /tmp/rp_dab_$1_$2 -o run --output-format csv -- python scripts/decode_ab.py --pmc > $out/pmc_$1_$2.log 2>&1 || exit $?
  find /tmp/rp_dab_$1_$2 -name '*counter_collection.csv' -exec cp {} $out/pmc_$1_$2.csv \;
done
cat $out/timing.jsonl
