# standalone conv backward: fused vs two kernels, weight-gradient grid 1 / 2 per CU
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
mkdir -p gpurun_out/ab
rm -f gpurun_out/ab/conv_standalone.txt
for m in 1 2 1 2; do echo "MLVAE_CONV_WG_MULT=$m" >> gpurun_out/ab/conv_standalone.txt; MLVAE_CONV_WG_MULT=$m timeout -k 10 120 python -u tools/conv_bench.py 100 >> gpurun_out/ab/conv_standalone.txt 2>&1 || exit 1; done
