import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
steps = float(sys.argv[2]) if len(sys.argv) > 2 else 1
tot = sum(float(r['TotalDurationNs']) for r in rows)
print(f"total {tot/1e6:.2f} ms  per-step {tot/1e6/steps:.3f} ms")
for r in rows[:int(sys.argv[3]) if len(sys.argv) > 3 else 20]:
    n = r['Name'].replace('(anonymous namespace)::', '')[:70]
    print(f"{n:70s} {int(r['Calls'])/steps:6.1f}/step {float(r['TotalDurationNs'])/1e3/steps:9.1f}us/step avg {float(r['AverageNs'])/1e3:8.1f}us {r['Percentage'][:5]}%")
