# densityopt throughput vs producer count (supershape renderer changes); the
# first run also warms MIOpen's kernel cache for the later ones.
set -e
mkdir -p gpurun_out/dopt
./pytorch-blender_amd/blendtorch/bin/supershapesim --bench 1000 > gpurun_out/dopt/supershapesim_bench.txt
for n in 4 4 8; do
  timeout -k 10 300 python examples/densityopt/densityopt.py --num-epochs 70 --instances $n --json gpurun_out/dopt/dopt_i$n.json > gpurun_out/dopt/dopt_i$n.log 2>&1
  tail -1 gpurun_out/dopt/dopt_i$n.log
done
cat gpurun_out/dopt/supershapesim_bench.txt
