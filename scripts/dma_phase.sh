# Does host->device DMA slow the consumer step, and does HOW it is ordered
# against the step matter?  profiles/r2/dma_phase.txt
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
mb() { timeout -k 10 200 "$@" > gpurun_out/mb.log 2>&1; grep "^{" gpurun_out/mb.log || { tail -20 gpurun_out/mb.log; exit 1; }; }
B="python scripts/disc_step_bench.py --only bf16-nhwc --graph on --iters 500 --cast fused --u8 --optim gfx950"
mb $B
for ph in none record start start_prev; do mb $B --dma 2 --dma-phase $ph; done
mb $B --dma 1 --dma-phase start
mb $B --dma 2 --dma-phase mid
