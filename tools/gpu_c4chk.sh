set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
mkdir -p gpurun_out/c4chk
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread -m gpu tests/test_gpu_conv.py tests/test_gpu_parity_bench.py -k "c4" > gpurun_out/c4chk/pytest.log 2>&1; rc=$?
grep -E "passed|failed|^\[c4|encoder.conv" gpurun_out/c4chk/pytest.log | tail -8
exit $rc
