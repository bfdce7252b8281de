#!/bin/bash
# Kernel trace of the streamed disc consumer step (bench.py --consumer disc), one step kernel by kernel.
# Usage: disc_trace.sh TAG [extra bench args]
set -u
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
tag=$1; shift
mkdir -p gpurun_out/trace_$tag
timeout -k 10 240 rocprofv3 --kernel-trace -d /tmp/dtr_$tag -o run --output-format csv -- python bench.py --consumer disc --steps 600 --warmup 50 "$@" > gpurun_out/trace_$tag/bench.log 2>&1 || { tail -5 gpurun_out/trace_$tag/bench.log; exit 1; }
python scripts/step_sequence.py /tmp/dtr_$tag --steps 300 > gpurun_out/trace_$tag/step_sequence.txt || exit 1
head -40 gpurun_out/trace_$tag/step_sequence.txt
grep -A40 'per kernel, summed' gpurun_out/trace_$tag/step_sequence.txt | head -30
