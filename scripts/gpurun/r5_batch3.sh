#!/bin/bash
# Round 5, GPU session 3: per-layer tile / staging sweep of the tap-gather GEMM
set -u
cd "$(dirname "$0")/../.."
O=gpurun_out/r5b3
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python scripts/conv_tile_sweep.py --iters 200 > $O/tile_sweep.jsonl 2>&1 || { tail -5 $O/tile_sweep.jsonl; exit 1; }
grep BEST $O/tile_sweep.jsonl
