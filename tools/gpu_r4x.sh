# m/n-contiguous staging with lane-invariant offsets precomputed (McLanes):
# GEMM / fp8 / step-parity tests; wgrad shapes VAR 0 vs 12 (same process); steps alternating
# A = libmlvae_base.so (before), B = new, C = new + MLVAE_GEMM_VAR=12 (ping-pong for the wgrads)
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
mkdir -p gpurun_out/ab
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_gemm_fast.py tests/test_gpu_fp8.py tests/test_gpu_step_parity.py > gpurun_out/r4x_tests.log 2>&1 && \
GEMM_FRAMES=128000 GEMM_VARS=0,12 GEMM_ONLY=wgrad timeout -k 10 200 python -u tools/gemm_bench.py > gpurun_out/ab/r4x_wgrad_vars.txt 2>&1 && \
rm -f gpurun_out/ab/summary_r4x.txt && \
for r in 1 2; do for c in c3 c5; do for v in A B C; do
  if [ $v = A ]; then L=$GRAFT_REPO_ROOT/ml-vae_amd/mlvae_hip/libmlvae_base.so; GV=0
  elif [ $v = B ]; then L=$GRAFT_REPO_ROOT/ml-vae_amd/mlvae_hip/libmlvae.so; GV=0
  else L=$GRAFT_REPO_ROOT/ml-vae_amd/mlvae_hip/libmlvae.so; GV=12; fi
  MLVAE_LIB_PATH=$L MLVAE_GEMM_VAR=$GV timeout -k 10 150 python -u bench.py --config $c --no-cpu-baseline --no-extra > gpurun_out/ab/r4x_${v}_${c}_$r.json 2>/dev/null || exit 1
  python3 -c "
import json
d=json.load(open('gpurun_out/ab/r4x_${v}_${c}_$r.json')); k=d['kernel_ms']
print('$v', '$c', $r, f\"{d['ms_per_step']:.3f} ms/step\", ' '.join(f'{n}={v:.3f}' for n, v in sorted(k.items())))
" >> gpurun_out/ab/summary_r4x.txt
done; done; done
