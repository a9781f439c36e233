set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp GEMM_FRAMES=128000
mkdir -p gpurun_out/gpmc
timeout -k 10 200 python -u tools/gemm_bench.py > gpurun_out/gpmc/bench.log 2>&1 || exit 1
export GEMM_ONLY="fwd proj" GEMM_MODES=1
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT --output-format csv -d gpurun_out/gpmc -o sq -- python3 tools/gemm_bench.py > gpurun_out/gpmc/sq.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d gpurun_out/gpmc -o tcc -- python3 tools/gemm_bench.py > gpurun_out/gpmc/tcc.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/gpmc -o fetch -- python3 tools/gemm_bench.py > gpurun_out/gpmc/fetch.log 2>&1 || exit 1
