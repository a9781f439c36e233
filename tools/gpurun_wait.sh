# Run one gpurun call, waiting out "no slot / box free" answers (nothing ran, nothing charged).
# Any answer where the command actually ran is final: no retry of a GPU step that ran.
# usage: bash tools/gpurun_wait.sh <timeout-seconds> '<command>' [log]
T=$1; CMD=$2; LOG=${3:-gpurun_out/call.txt}
mkdir -p gpurun_out
for i in $(seq 1 30); do
  /usr/local/graft/bin/gpurun --timeout "$T" -- "$CMD" > "$LOG" 2>&1
  rc=$?
  if [ $rc -eq 3 ] || grep -q "status=transient rc=None" "$LOG"; then
    echo "[wait] attempt $i: no box yet (rc=$rc); sleeping" >> "$LOG.wait"
    sleep 60
    continue
  fi
  break
done
tail -25 "$LOG"
exit $rc
