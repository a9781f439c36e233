# Round-6 traffic refresh: per config a kernel trace (launch order for the role tables) and the two
# PMC passes (FETCH_SIZE, WRITE_SIZE), each under its own limit; post-processed on the host
# (tools/pmc_summary.py).  configs: $CFGS (default c3 c5 c5bf16 c2 c4)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
for CFG in ${CFGS:-c3 c5 c5bf16 c2 c4}; do
  O=gpurun_out/pmc6/$CFG
  mkdir -p $O
  timeout -s KILL 150 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o trace -- \
    python3 -u bench.py --config $CFG --steps 3 --warmup 1 --no-cpu-baseline --no-extra > $O/trace.log 2>&1 || exit 1
  timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O -o fetch -- \
    python3 -u bench.py --config $CFG --steps 3 --warmup 1 --no-cpu-baseline --no-extra > $O/fetch.log 2>&1 || exit 1
  timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O -o write -- \
    python3 -u bench.py --config $CFG --steps 3 --warmup 1 --no-cpu-baseline --no-extra > $O/write.log 2>&1 || exit 1
  echo "$CFG done: $(tail -1 $O/trace.log | cut -c1-120)"
done
