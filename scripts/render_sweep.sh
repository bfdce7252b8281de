# Producer-count sweep after the incremental/SIMD renderer: throughput and the
# CPU it costs (cgroup usage over the timed region), long runs for stable numbers.
set -e
mkdir -p gpurun_out/render
B=pytorch-blender_amd/blendtorch/bin/cubesim
$B --bench 2000 --mode rgba > gpurun_out/render/cubesim_bench_rgba.json
for p in 2 3 4 6 8; do
  timeout -k 10 180 python bench.py --steps 20000 --warmup 200 --producers $p > gpurun_out/render/long_p$p.json 2> gpurun_out/render/long_p$p.err
done
BLENDTORCH_FULL_RENDER=1 timeout -k 10 180 python bench.py --steps 20000 --warmup 200 --producers 4 > gpurun_out/render/long_p4_full.json 2> gpurun_out/render/long_p4_full.err
timeout -k 10 180 python bench.py --steps 20000 --warmup 200 > gpurun_out/render/long_default.json 2> gpurun_out/render/long_default.err
