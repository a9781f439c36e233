"""Kernel stats and one step's timeline from a rocprofv3 rocpd SQLite database.

usage: python tools/rocpd_timeline.py <run_results.db> [steps=23] [step_index_from_end=2]
Steps are delimited by the Adam kernel (one per training step)."""
import collections
import sqlite3
import sys


def short(name):
    return name.replace("(anonymous namespace)::", "").split("(")[0][:60]


def main(path, steps=23, back=2):
    c = sqlite3.connect(path)
    rows = c.execute("select name, start, end, queue_id, grid_x from kernels order by start").fetchall()
    agg = collections.defaultdict(lambda: [0, 0])
    for n, s, e, q, g in rows:
        agg[short(n)][0] += 1
        agg[short(n)][1] += e - s
    tot = sum(v[1] for v in agg.values())
    print(f"total {tot / 1e6:.2f} ms over {steps} steps: {tot / 1e6 / steps:.3f} ms/step of kernel time")
    for n, (k, d) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:30]:
        print(f"{n:60s} {k / steps:6.1f}/step {d / 1e3 / steps:9.1f}us/step avg {d / k / 1e3:8.1f}us {100 * d / tot:5.1f}%")
    adam = [i for i, r in enumerate(rows) if "adam_kernel" in r[0]]
    if len(adam) > back:
        i0, i1 = adam[-back - 1] + 1, adam[-back] + 1
        t0 = rows[i0][1]
        print("\none step:")
        for n, s, e, q, g in rows[i0:i1]:
            print(f"q{q:>2} {(s - t0) / 1e3:9.1f} {(e - t0) / 1e3:9.1f} {(e - s) / 1e3:8.1f}us  grid {g:>7} {short(n)}")
        print(f"step span {(rows[i1 - 1][2] - t0) / 1e3:.1f} us")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 23,
         int(sys.argv[3]) if len(sys.argv) > 3 else 2)
