set -u
cd $GRAFT_REPO_ROOT
for d in 0 1 2 4; do
  timeout -k 10 200 python scripts/disc_step_bench.py --only bf16-nhwc --graph on --iters 500 --dma $d 2>&1 | grep '^{' || exit 1
done
