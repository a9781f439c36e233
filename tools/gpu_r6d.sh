set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r6d
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 200 python -u -m pytest tests/test_gpu_skinny.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r6d/skinny.log 2>&1 || exit 1
for i in 1 2; do
  for lib in abl/libmlvae_pre_tn.so ml-vae_amd/mlvae_hip/libmlvae.so; do
    for c in c5 c5bf16 c2; do
      echo "$lib $c $(MLVAE_LIB_PATH=$GRAFT_REPO_ROOT/$lib timeout -k 10 120 python bench.py --config $c --steps 20 --warmup 3 --no-cpu-baseline --no-extra 2>/dev/null | python -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"])')" >> gpurun_out/r6d/ab.txt || exit 1
    done
  done
done
export MLVAE_LIB_PATH=$GRAFT_REPO_ROOT/ml-vae_amd/mlvae_hip/libmlvae_diag.so
STAMPS_TAG=_r6 bash tools/gpu_stamps.sh
