# same-box A/B of the current library against the round-6 start build (abl/libmlvae_r6start.so: built from 6b841cc into abl/ first; not kept in the tree)
# at c3 and the fp8 / bf16 c5 shard
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
REPS=2 bash tools/gpu_run.sh - "c3 c5 c5bf16" abr6 "MLVAE_NONE=0" "MLVAE_LIB_PATH=$GRAFT_REPO_ROOT/abl/libmlvae_r6start.so"
