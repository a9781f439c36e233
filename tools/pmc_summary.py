"""Per-kernel HBM traffic per launch from two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE).

usage: python tools/pmc_summary.py <fetch counter_collection.csv> <write counter_collection.csv> <out.json> <config>

The result is merged into out.json under the bench config's name (c2, c3, ...): bench.py reads
profiles/pmc_traffic.json[config][kernel] for its roofline "traffic" fields.

Both counters are reported in KB.  MI355X_MICROARCH.md (HBM section): on gfx950 FETCH_SIZE
counts exactly half of the bytes of wide coalesced streaming reads, so the read bytes are
taken as 2 x FETCH_SIZE; WRITE_SIZE is exact for 16-B streaming stores.  hbm_bytes_per_launch =
2*FETCH + WRITE (the raw values are kept next to it)."""
import collections
import csv
import json
import os
import sys


def per_kernel(path):
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        agg[r["Kernel_Name"]].append(float(r["Counter_Value"]) * 1024.0)
    return agg


def short(name):
    n = name.replace("(anonymous namespace)::", "")
    for frag, key in (("lstm_bwd", "lstm_bwd"), ("lstm_fwd", "lstm_fwd"), ("heads_kernel", "heads"),
                      ("encoder_fwd_kernel", "encoder_fwd"), ("encoder_bwd_kernel", "encoder_bwd"),
                      ("conv_wgrad_kernel", "conv_wgrad"), ("gemm256_kernel<true, true, 8>", "gemm_fp8")):
        if frag in n:
            return key
    if "conv_kernel" in n:  # forward layers / input gradient (csrc/conv.hip)
        return "conv_dgrad" if "true>" in n else "conv_fwd_layer"
    return n.split("(")[0]


def main(fetch_csv, write_csv, out, config):
    f, w = per_kernel(fetch_csv), per_kernel(write_csv)
    res = {}
    for name in set(f) | set(w):
        fv, wv = f.get(name, [0.0]), w.get(name, [0.0])
        fetch = sum(fv) / len(fv)
        write = sum(wv) / len(wv)
        key = short(name)
        if key in res and res[key]["launches"] >= len(fv):
            continue
        res[key] = {"kernel": name, "launches": len(fv), "fetch_size_bytes_raw": fetch,
                    "write_size_bytes": write, "read_bytes_corrected": 2 * fetch,
                    "hbm_bytes_per_launch": 2 * fetch + write}
    res = dict(sorted(res.items(), key=lambda kv: -kv[1]["hbm_bytes_per_launch"]))
    try:
        with open(out) as fh:
            allres = json.load(fh)
    except (OSError, ValueError):
        allres = {}
    # where the numbers came from (bench.py cites it next to every "traffic" it reports)
    tag = os.environ.get("PMC_TAG", "")
    res["_source"] = {"fetch_csv": os.path.basename(fetch_csv), "write_csv": os.path.basename(write_csv),
                      "tag": tag, "committed_as": f"profiles/pmc_{tag or config}_{{fetch,write}}.csv"}
    allres[config] = res
    json.dump(allres, open(out, "w"), indent=1)
    for k, v in [kv for kv in res.items() if not kv[0].startswith('_')][:10]:
        print(f"{k:40s} launches {v['launches']:3d}  read {v['read_bytes_corrected'] / 1e6:9.1f} MB  "
              f"write {v['write_size_bytes'] / 1e6:9.1f} MB")


if __name__ == "__main__":
    main(*sys.argv[1:5])
