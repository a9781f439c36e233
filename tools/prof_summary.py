"""Per-kernel summary of a rocprofv3 --kernel-trace --stats CSV (kernel_stats.csv).

    python tools/prof_summary.py <kernel_stats.csv> <steps traced> [top N]

`steps traced` is the number of train steps the profiled command ran (warmup + timed): the
totals in the CSV cover all of them, and the per-step columns divide by it.  There is no
default -- a summary without it would label whole-trace totals as per-step figures."""
import csv
import sys

if len(sys.argv) < 3:
    sys.exit(__doc__)
rows = list(csv.DictReader(open(sys.argv[1])))
steps = float(sys.argv[2])
top = int(sys.argv[3]) if len(sys.argv) > 3 else 20
tot = sum(float(r['TotalDurationNs']) for r in rows)
print(f"kernel time over the trace {tot / 1e6:.2f} ms in {steps:g} steps = {tot / 1e6 / steps:.3f} ms per step")
for r in rows[:top]:
    n = r['Name'].replace('(anonymous namespace)::', '')[:70]
    print(f"{n:70s} {int(r['Calls']) / steps:6.1f} launches/step {float(r['TotalDurationNs']) / 1e3 / steps:9.1f} us/step "
          f"avg {float(r['AverageNs']) / 1e3:8.1f} us/launch {r['Percentage'][:5]}%")
