#!/bin/bash
# Round 6, GPU session 26: the data-parallel code paths after the update took the last slice reduce
# (a collective follows the backward there, so the reduce keeps its launch; the schedule rides early):
# disc with a 1-rank RCCL group (--force-pg), and 2 gloo ranks sharing the one GPU.
set -u
cd "$(dirname "$0")/../.."
O=gpurun_out/r6b26
mkdir -p $O
export TMPDIR=/tmp
trap 'du -sh gpurun_out' EXIT
timeout -k 10 240 python bench.py --consumer disc --force-pg --steps 1000 > $O/disc_forcepg.log 2>&1 || { tail -5 $O/disc_forcepg.log; exit 1; }
grep '^{' $O/disc_forcepg.log | tee $O/disc_forcepg.jsonl | cut -c1-200
timeout -k 10 240 python bench.py --consumer disc --steps 1000 > $O/disc.log 2>&1 || { tail -5 $O/disc.log; exit 1; }
grep '^{' $O/disc.log | tee $O/disc.jsonl | cut -c1-200
timeout -k 10 300 python bench.py --consumer disc --gpus 2 --backend gloo --steps 300 > $O/disc_gloo2.log 2>&1 || { tail -8 $O/disc_gloo2.log; exit 1; }
grep '^{' $O/disc_gloo2.log | tee $O/disc_gloo2.jsonl | cut -c1-240
