#!/bin/bash
# One gpurun session: GPU tests, smoke, bench, profile.  Stops at the first
# GPU fault / abort / timeout (exit codes other than 0 = ok, 1 = test failure).
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
cleanup() { find gpurun_out -type f -size +8M -print -delete; du -sh gpurun_out; }
trap cleanup EXIT
ok() { local rc=$1; [ "$rc" -eq 0 ] || [ "$rc" -eq 1 ]; }
echo "== host: nproc=$(nproc) affinity=$(python -c 'import os;print(len(os.sched_getaffinity(0)))') cpu.max=$(cat /sys/fs/cgroup/cpu.max 2>/dev/null)" | tee gpurun_out/host.txt
timeout -k 10 240 python -c "import sys; sys.path.insert(0,'.'); import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || { echo build failed; tail -20 gpurun_out/build.log; exit 2; }
for step in "$@"; do
  case "$step" in
    tests) timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -5 gpurun_out/pytest_gpu.log;;
    smoke) timeout -k 10 200 python -c "import sys; sys.path.insert(0,'.'); import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?; tail -3 gpurun_out/smoke.log;;
    bench) timeout -k 10 300 python bench.py > gpurun_out/bench.log 2>&1; rc=$?; tail -3 gpurun_out/bench.log;;
    bench:*) a="${step#bench:}"; timeout -k 10 300 python bench.py ${a//,/ } >> gpurun_out/bench_sweep.log 2>&1; rc=$?; tail -1 gpurun_out/bench_sweep.log;;
    prof) timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/rp_prof -o run --output-format csv -- python bench.py --steps 300 --warmup 20 > gpurun_out/prof.log 2>&1; rc=$?; tail -2 gpurun_out/prof.log
          mkdir -p gpurun_out/prof && find /tmp/rp_prof -name '*stats.csv' -exec cp {} gpurun_out/prof/ \;;;
    prof:*) a="${step#prof:}"; tag=$(echo "$a" | tr -c 'a-zA-Z0-9\n' '_'); timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/rp_prof_$tag -o run --output-format csv -- python bench.py --steps 300 --warmup 20 ${a//,/ } > gpurun_out/prof_$tag.log 2>&1; rc=$?; grep '^{' gpurun_out/prof_$tag.log | cut -c1-200
          mkdir -p gpurun_out/prof_$tag && find /tmp/rp_prof_$tag -name '*stats.csv' -exec cp {} gpurun_out/prof_$tag/ \;;;
    cpmc) for pass in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES" "FETCH_SIZE" "WRITE_SIZE GRBM_GUI_ACTIVE"; do
            n=$((${n:-0}+1))
            timeout -s KILL 90 rocprofv3 --pmc $pass --kernel-trace -d /tmp/rp_cpmc$n -o run --output-format csv -- python scripts/consumer_pmc.py > gpurun_out/cpmc$n.log 2>&1; rc=$?
            mkdir -p gpurun_out/cpmc && find /tmp/rp_cpmc$n -name '*counter_collection.csv' -exec cp {} gpurun_out/cpmc/pass${n}_counters.csv \;
            rm -f gpurun_out/cpmc$n.log
            ok $rc || { echo "cpmc pass $n rc=$rc"; exit $rc; }
          done;;
    dstep) timeout -k 10 200 python scripts/disc_step_bench.py --only bf16-nhwc > gpurun_out/disc_step.log 2>&1; rc=$?; grep '^{' gpurun_out/disc_step.log;;
    kbench) timeout -k 10 200 python scripts/kernel_bench.py --json gpurun_out/kernel_bench.json > gpurun_out/kernel_bench.log 2>&1; rc=$?; cat gpurun_out/kernel_bench.log;;
    kprof) timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/rp_kprof -o run --output-format csv -- python scripts/kernel_bench.py --iters 50 > gpurun_out/kprof.log 2>&1; rc=$?
          mkdir -p gpurun_out/kprof && find /tmp/rp_kprof -name '*stats.csv' -exec cp {} gpurun_out/kprof/ \;;;
    kpmc) for pass in "SQ_INSTS_MFMA SQ_INSTS_VALU_MFMA_F32 SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVES SQ_INSTS_VALU SQ_BUSY_CYCLES" "FETCH_SIZE" "WRITE_SIZE GRBM_GUI_ACTIVE"; do
            n=$((${n:-0}+1))
            timeout -k 10 240 rocprofv3 --pmc $pass --kernel-trace -d /tmp/rp_kpmc$n -o run --output-format csv -- python scripts/kernel_pmc.py > gpurun_out/kpmc$n.log 2>&1; rc=$?
            mkdir -p gpurun_out/kpmc && find /tmp/rp_kpmc$n -name '*counter_collection.csv' -exec cp {} gpurun_out/kpmc/pass${n}_counters.csv \;
            ok $rc || { echo "kpmc pass $n rc=$rc"; exit $rc; }
          done;;
    rl) timeout -k 10 200 python benchmarks/bench_rl.py --envs 8 --steps 5000 > gpurun_out/bench_rl.log 2>&1; rc=$?; tail -1 gpurun_out/bench_rl.log
        timeout -k 10 200 python benchmarks/bench_rl.py --envs 1 --steps 5000 >> gpurun_out/bench_rl.log 2>&1; rc=$?; tail -1 gpurun_out/bench_rl.log;;
    dopt) timeout -k 10 300 python examples/densityopt/densityopt.py --num-epochs 70 --json gpurun_out/densityopt.json > gpurun_out/densityopt.log 2>&1; rc=$?; tail -2 gpurun_out/densityopt.log;;
    ksweep) for mg in ${KSWEEP_GRIDS:-1024 2048 4096 16384}; do for pm in ${KSWEEP_PPT:-1 2 4}; do
            BT_DECODE_MAXGRID=$mg BT_DECODE_PPT_MULT=$pm timeout -k 10 120 python scripts/kernel_bench.py --only decode --tag "grid=$mg ppt_mult=$pm" >> gpurun_out/ksweep.log 2>&1 || { rc=$?; break 2; }
          done; done; rc=${rc:-0}; grep -o "grid=.*speedup" gpurun_out/ksweep.log | sed "s/'torch_eager_us.*//" ;;
    trace) BLENDTORCH_ROCTX=1 timeout -k 10 300 rocprofv3 --marker-trace --kernel-trace --stats -d /tmp/rp_trace -o run --output-format csv -- python bench.py --steps 300 --warmup 20 > gpurun_out/trace.log 2>&1; rc=$?; tail -2 gpurun_out/trace.log
          mkdir -p gpurun_out/trace && find /tmp/rp_trace -name '*stats.csv' -exec cp {} gpurun_out/trace/ \;;;
    dist1) timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29555 bench.py --gpus 1 --steps 500 --warmup 20 > gpurun_out/dist1.log 2>&1; rc=$?; grep '^{' gpurun_out/dist1.log;
           timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29556 bench.py --gpus 1 --steps 300 --warmup 20 --consumer disc >> gpurun_out/dist1.log 2>&1; rc=$?; grep '^{' gpurun_out/dist1.log | tail -1;;
    sup2) timeout -k 10 300 python bench.py --gpus 2 --backend gloo --steps 1000 --warmup 20 > gpurun_out/sup2.log 2>&1; rc=$?; grep '^{' gpurun_out/sup2.log | cut -c1-600;;
    sup2:*) a="${step#sup2:}"; timeout -k 10 300 python bench.py --gpus 2 --backend gloo ${a//,/ } >> gpurun_out/sup2.log 2>&1; rc=$?; grep '^{' gpurun_out/sup2.log | tail -1 | cut -c1-600;;
    supn:*) a="${step#supn:}"; n="${a%%,*}"; rest="${a#*,}"; timeout -k 10 400 python bench.py --gpus $n --backend gloo ${rest//,/ } >> gpurun_out/supn.log 2>&1; rc=$?; grep '^{' gpurun_out/supn.log | tail -1 | cut -c1-400;;
    gtests:*) a="${step#gtests:}"; timeout -k 10 500 python -u -m pytest ${a//,/ } -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu_sel.log 2>&1; rc=$?; grep -E "PASS|FAIL|ERROR|passed|failed" gpurun_out/pytest_gpu_sel.log | tail -30;;
    b:*) a="${step#b:}"; tag=$(echo "$a" | tr -c 'a-zA-Z0-9\n' '_' | cut -c1-60); timeout -k 10 300 python bench.py ${a//,/ } > gpurun_out/b_$tag.log 2>&1; rc=$?; grep '^{' gpurun_out/b_$tag.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$a', '->', d['value'], d['unit'], d['ms_per_step'], 'ms', d.get('h2d_gbytes_per_s'), 'GB/s', d['config'].get('consumer_step'), d.get('world_size_seen'))" || tail -5 gpurun_out/b_$tag.log;;
    ktrace:*) a="${step#ktrace:}"; tag=$(echo "$a" | tr -c 'a-zA-Z0-9\n' '_' | cut -c1-50); timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d /tmp/rp_kt_$tag -o run --output-format csv -- python bench.py ${a//,/ } > gpurun_out/kt_$tag.log 2>&1; rc=$?; grep '^{' gpurun_out/kt_$tag.log | cut -c1-300
          python scripts/trace_timeline.py /tmp/rp_kt_$tag --last ${KT_LAST:-20000} > gpurun_out/kt_$tag.txt 2>&1; cat gpurun_out/kt_$tag.txt;;
    ktstep) timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/rp_ktstep -o run --output-format csv -- python scripts/disc_step_bench.py --only bf16-nhwc --graph on --iters 300 > gpurun_out/ktstep.log 2>&1; rc=$?; grep '^{' gpurun_out/ktstep.log
          python scripts/trace_timeline.py /tmp/rp_ktstep --last ${KT_LAST:-20000} > gpurun_out/ktstep.txt 2>&1; cat gpurun_out/ktstep.txt;;
    replay2) for args in "--batch 8" "--batch 64 --steps 500" "--batch 8 --graph" "--batch 64 --steps 500 --graph" "--batch 8 --sampler legacy" "--batch 64 --steps 500 --sampler legacy" "--batch 64 --steps 500 --dtype bfloat16"; do
            timeout -k 10 200 python benchmarks/bench_replay.py $args >> gpurun_out/replay2.log 2>&1 || { rc=$?; break; }
          done; rc=${rc:-0}; grep '^{' gpurun_out/replay2.log | python -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print(d['sampler'], 'B', d['batch'], 'graph', d['graph'], d['dtype'], d['us_per_batch'], 'us', d['effective_tbps'], 'TB/s', d['value'], 'img/s')";;
    rpmc) for pass in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES" "FETCH_SIZE" "WRITE_SIZE GRBM_GUI_ACTIVE"; do
            n=$((${n:-0}+1))
            timeout -s KILL 90 rocprofv3 --pmc $pass --kernel-trace -d /tmp/rp_rpmc$n -o run --output-format csv -- python scripts/replay_pmc.py > gpurun_out/rpmc$n.log 2>&1; rc=$?
            mkdir -p gpurun_out/rpmc && find /tmp/rp_rpmc$n -name '*counter_collection.csv' -exec cp {} gpurun_out/rpmc/pass${n}_counters.csv \;
            ok $rc || { echo "rpmc pass $n rc=$rc"; exit $rc; }
          done;;
    sweep) timeout -k 10 900 python benchmarks/sweep.py --out gpurun_out/sweep.jsonl > gpurun_out/sweep.log 2>&1; rc=$?; python -c "
import json
for l in open('gpurun_out/sweep.jsonl'):
    d=json.loads(l); print(d['mode'], d['producers'], d['images_per_s'], d['sec_per_image'], d['ratio_vs_reference_row'], d['h2d_gbytes_per_s'])";;
    rtrace) timeout -k 10 200 rocprofv3 --kernel-trace --stats -d /tmp/rp_rtrace -o run --output-format csv -- python benchmarks/bench_replay.py --batch 8 --frames 1024 --steps 500 > gpurun_out/rtrace.log 2>&1; rc=$?
          mkdir -p gpurun_out/rtrace && find /tmp/rp_rtrace -name '*kernel_stats.csv' -exec cp {} gpurun_out/rtrace/ \; ; head -5 gpurun_out/rtrace/*kernel_stats.csv | cut -c1-220;;
    mtrace:*) a="${step#mtrace:}"; BLENDTORCH_ROCTX=1 timeout -k 10 300 rocprofv3 --marker-trace --kernel-trace -d /tmp/rp_mt -o run --output-format csv -- python bench.py ${a//,/ } > gpurun_out/mtrace.log 2>&1; rc=$?; grep '^{' gpurun_out/mtrace.log | cut -c1-200
          python scripts/marker_summary.py /tmp/rp_mt > gpurun_out/mtrace.txt 2>&1; cat gpurun_out/mtrace.txt
          python scripts/trace_timeline.py /tmp/rp_mt --last 20000 > gpurun_out/mtrace_k.txt 2>&1; head -30 gpurun_out/mtrace_k.txt;;
    short) timeout -k 10 200 python bench.py --steps 20 --warmup 5 > gpurun_out/short.log 2>&1; rc=$?; grep '^{' gpurun_out/short.log;;
    dist2gloo) timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29557 bench.py --gpus 2 --backend gloo --steps 1000 --warmup 20 > gpurun_out/dist2gloo.log 2>&1; rc=$?; grep '^{' gpurun_out/dist2gloo.log;;
    replay) timeout -k 10 200 python benchmarks/bench_replay.py > gpurun_out/replay.log 2>&1 && timeout -k 10 200 python benchmarks/bench_replay.py --batch 64 --steps 500 >> gpurun_out/replay.log 2>&1 && timeout -k 10 200 python benchmarks/bench_replay.py --graph >> gpurun_out/replay.log 2>&1 && timeout -k 10 200 python benchmarks/bench_replay.py --graph --batch 64 --steps 500 >> gpurun_out/replay.log 2>&1 && timeout -k 10 200 python benchmarks/bench_replay.py --fill producers --frames 2048 --batch 64 --steps 500 >> gpurun_out/replay.log 2>&1; rc=$?; cat gpurun_out/replay.log | grep '^{';;
    dpmc) timeout -k 10 120 rocprofv3 --pmc TCC_EA0_RDREQ_IO_32B_sum TCC_EA0_RDREQ_IO_CREDIT_STALL_sum TCC_EA0_RDREQ_DRAM_32B_sum --kernel-trace -d /tmp/rp_dpmc1 -o run --output-format csv -- python scripts/direct_pmc.py > gpurun_out/dpmc1.log 2>&1; rc=$?
          mkdir -p gpurun_out/dpmc && find /tmp/rp_dpmc1 -name '*counter_collection.csv' -exec cp {} gpurun_out/dpmc/pass1_counters.csv \;
          ok $rc || { echo "dpmc pass1 rc=$rc"; exit $rc; }
          timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE --kernel-trace -d /tmp/rp_dpmc2 -o run --output-format csv -- python scripts/direct_pmc.py > gpurun_out/dpmc2.log 2>&1; rc=$?
          find /tmp/rp_dpmc2 -name '*counter_collection.csv' -exec cp {} gpurun_out/dpmc/pass2_counters.csv \;;;
    usweep) for bsz in 8 64; do for u in 1 2; do for mg in 2048 4096 8192; do
            BT_DECODE_UNROLL=$u BT_DECODE_MAXGRID=$mg timeout -k 10 120 python scripts/kernel_bench.py --only decode --no-ref --batch $bsz --iters 100 --tag "B=$bsz unroll=$u grid=$mg" >> gpurun_out/usweep.log 2>&1 || { rc=$?; break 3; }
          done; done; done; rc=${rc:-0}; grep -o "B=.*GBps': [0-9.]*" gpurun_out/usweep.log;;
    train) timeout -k 10 300 python examples/datagen/train_keypoints.py --steps 400 --json gpurun_out/train_keypoints.json > gpurun_out/train.log 2>&1; rc=$?; grep '^{' gpurun_out/train.log;;
    dist2pool) timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29558 bench.py --gpus 2 --backend gloo --dist pool --steps 1000 --warmup 20 > gpurun_out/dist2pool.log 2>&1; rc=$?; grep '^{' gpurun_out/dist2pool.log;;
    trainprof) timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/rp_train -o run --output-format csv -- python examples/datagen/train_keypoints.py --steps 60 > gpurun_out/trainprof.log 2>&1; rc=$?; grep '^{' gpurun_out/trainprof.log
          mkdir -p gpurun_out/trainprof && find /tmp/rp_train -name '*kernel_stats.csv' -exec cp {} gpurun_out/trainprof/ \;;;
    rlsweep) for cfg in ${RL_CFGS:-"8 tcp 0" "8 ipc 0" "32 ipc 0" "1 ipc 0"}; do set -- $cfg
            timeout -k 10 200 python benchmarks/bench_rl.py --envs $1 --proto $2 --io-threads $3 --steps 4000 >> gpurun_out/rlsweep.log 2>&1 || { rc=$?; break; }
          done; rc=${rc:-0}; grep '^{' gpurun_out/rlsweep.log;;
    train2) BLENDTORCH_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29559 examples/datagen/train_keypoints.py --steps 150 --batch 16 --producers 4 > gpurun_out/train2.log 2>&1; rc=$?; grep '^{' gpurun_out/train2.log;;
    h2d) timeout -k 10 120 python -c "
import sys; sys.path.insert(0,'pytorch-blender_amd')
import torch; from blendtorch import ops; e=ops.hip_ext()
for k in ('hostmalloc','register','pageable'):
    for chunks in (1,8):
        print(k, 'chunks', chunks, round(e.bench_h2d(k, 1228800, 200, chunks),2), 'GB/s', flush=True)
" > gpurun_out/h2d.log 2>&1; rc=$?; cat gpurun_out/h2d.log;;
    f2d) timeout -k 10 180 python -c "
import sys; sys.path.insert(0,'pytorch-blender_amd')
import torch; from blendtorch import ops; e=ops.hip_ext()
import os
B = int(os.environ.get('F2D_B', '8'))
for cin in (4,):
  for kind in ('register', 'register_thp', 'hostmalloc'):
    for mode, grids in (('copy', (0,)), ('direct', (0, 4096))):
        for g in grids:
            us, gbs, stale = e.bench_frames_to_device(mode, kind, B, 480, 640, cin, 300, g)
            print(f'B={B} cin={cin} {kind:10s} {mode:6s} grid={g:5d} {us:8.1f} us/batch {gbs:6.1f} GB/s stale={stale}', flush=True)
" > gpurun_out/f2d.log 2>&1; rc=$?; cat gpurun_out/f2d.log;;
    *) echo "unknown step $step"; rc=2;;
  esac
  echo "== step $step rc=$rc"
  ok $rc || exit $rc
done
