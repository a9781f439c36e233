"""Print one training step's kernel timeline from a rocprofv3 kernel_trace.csv.

usage: python tools/trace_step.py <run_kernel_trace.csv> [step_index_from_end=2]
Steps are delimited by the Adam kernel (one per step)."""
import csv
import sys


def main(path, back=2):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    adam = [i for i, r in enumerate(rows) if "adam_kernel" in r["Kernel_Name"]]
    i0, i1 = adam[-back - 1] + 1, adam[-back] + 1
    t0 = int(rows[i0]["Start_Timestamp"])
    for r in rows[i0:i1]:
        s, e = int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0
        name = r["Kernel_Name"].replace("(anonymous namespace)::", "")
        name = name.split("(")[0][:48]
        print(f"q{r['Queue_Id']:>2} {s / 1e3:9.1f} {e / 1e3:9.1f} {(e - s) / 1e3:8.1f}us  grid {r['Grid_Size_X']:>7} {name}")
    print(f"step span {(int(rows[i1 - 1]['End_Timestamp']) - t0) / 1e3:.1f} us")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 2)
