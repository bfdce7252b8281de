set -u
cd $GRAFT_REPO_ROOT
bash scripts/gpurun/r2_disc.sh || exit 1
bash scripts/disc_ktrace.sh
