cd $GRAFT_REPO_ROOT
export PYTHONDONTWRITEBYTECODE=1
mkdir -p gpurun_out/dbg
rm -f gpurun_out/dbg/fwd_err.txt
for args in "--B 64 --T 6 --mode 2048" "--B 16 --T 4 --mode 6144"; do
  timeout -k 10 60 python -u tools/dbg_fwd_err.py $args >> gpurun_out/dbg/fwd_err.txt 2>&1 || exit 1
done
