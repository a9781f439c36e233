"""Per-launch HBM traffic of the train step's kernels, by ROLE, from two rocprofv3 --pmc passes
(FETCH_SIZE, WRITE_SIZE) over a short bench run.

usage: python tools/pmc_summary.py <fetch counter_collection.csv> <write counter_collection.csv> <out.json> <config>

Round 5: one kernel instance serves several roles in a step -- the layer-0
forward recurrence (its fused z projection) and the layer-1 one are different instances, but the
256x256 GEMM instance <true, true, 12> runs the layer-1 projection, the heads' P1 and dY and the
layer-1 dgrad.  The dispatches are therefore split into steps (one adam_kernel per step) and each
dispatch is named by its kernel and its occurrence within the step (ROLES below: the engine's
fixed launch order, engine.py).  A step whose count of a kernel differs from the table (the fp8
mode's first step runs a bf16 dgrad) is skipped for that kernel.  The result is merged into
out.json[config][role]; bench.py sets every "traffic" beside the algorithmic bytes of the same
launch(es).

Both counters are reported in KB.  MI355X_MICROARCH.md (HBM section): on gfx950 FETCH_SIZE
counts exactly half of the bytes of wide coalesced streaming reads, so the read bytes are taken
as 2 x FETCH_SIZE; WRITE_SIZE is exact for 16-B streaming stores.  hbm_bytes_per_launch =
2*FETCH + WRITE (the raw values are kept next to it)."""
import collections
import csv
import json
import os
import sys

# kernel-name fragment -> role of its k-th dispatch within a step (engine.py launch order; the
# round-6 main loops: VAR 16 k-contiguous, VAR 18 m/n-contiguous unshifted, VAR 0 time-shifted dW_hh,
# fp8 VAR 8 k-contiguous and VAR 9 m/n-contiguous; the time-shifted VAR 0 no longer runs)
_COMMON = [
    ("lstm_fwd_wide_kernel", ["lstm_fwd_l0", "lstm_fwd_l1"]),
    ("lstm_bwd_wide_kernel", ["lstm_bwd_l1", "lstm_bwd_l0"]),
    ("heads_mid_kernel", ["heads_mid"]),
    ("encoder_fwd_kernel", ["encoder_fwd"]),
    ("encoder_bwd_kernel", ["encoder_bwd"]),
]
ROLES_BF16 = _COMMON + [   # c3: from 64K frames the heads' products run on the 128-row heads_nt kernel
    ("gemm256_kernel<true, true, 16>", ["proj_l1", "dgrad_l1"]),
    ("heads_nt_kernel<true", ["heads_p1"]),
    ("heads_nt_kernel<false", ["heads_dy"]),
    # dW_hh_l1: the utterance-boundary terms, then the unshifted product; dW_hh_l0 on the
    # pre-shifted h (engine _whh_bf16 / yb_prev)
    ("gemm256_kernel<false, false, 18>", ["heads_dw1", "wgrad_ih_l1", "wgrad_hh_l1_bnd", "wgrad_hh_l1",
                                          "wgrad_hh_l0"]),
    ("skinny_dzw_kernel", ["skinny_dzw"]),
]
ROLES_C4 = _COMMON + [     # Conv1d encoder: layer 0 has its own 256-wide input projection / dW_ih
    ("gemm256_kernel<true, true, 16>", ["proj_l1", "dgrad_l1"]),
    ("heads_nt_kernel<true", ["heads_p1"]),
    ("heads_nt_kernel<false", ["heads_dy"]),
    ("gemm256_kernel<false, false, 18>", ["heads_dw1", "wgrad_ih_l1", "wgrad_hh_l1_bnd", "wgrad_hh_l1",
                                          "wgrad_ih_l0", "wgrad_hh_l0"]),
    ("conv_kernel<4, false>", ["conv_fwd_l1", "conv_fwd_l2"]),
    ("conv_kernel<4, true>", ["conv_dgrad"]),
    ("conv_wgrad_kernel", ["conv_wgrad_l2", "conv_wgrad_l1"]),
]
# below 64K frames (c2, the c5 shard in bf16, c3h): P1 on heads_nt, dY on the 256² GEMM
ROLES_SMALL = _COMMON + [
    ("gemm256_kernel<true, true, 16>", ["proj_l1", "heads_dy", "dgrad_l1"]),
    ("heads_nt_kernel<true", ["heads_p1"]),
    ("gemm256_kernel<false, false, 18>", ["heads_dw1", "wgrad_ih_l1", "wgrad_hh_l1_bnd", "wgrad_hh_l1",
                                          "wgrad_hh_l0"]),
    ("skinny_nt_lds_kernel<2, false>", ["skinny_dz"]),
    ("skinny_tn_kernel<3, false>", ["skinny_dwih_l0"]),
]
ROLES_FP8 = _COMMON + [    # c5: e4m3 operands from the second step on (the first step's bf16 forms skip)
    ("gemm256_kernel<true, true, 8>", ["proj_l1", "dgrad_l1"]),
    ("heads_nt_kernel<true", ["heads_p1"]),
    ("gemm256_kernel<true, true, 16>", ["heads_dy"]),
    ("gemm256_kernel<false, false, 18>", ["heads_dw1"]),
    ("gemm256_kernel<false, false, 9>", ["wgrad_ih_l1", "wgrad_hh_l1", "wgrad_hh_l0"]),
    ("skinny_nt_lds_kernel<2, true>", ["skinny_dz"]),
    ("skinny_tn_kernel<3, true>", ["skinny_dwih_l0"]),
]
ROLES = {"c5": ROLES_FP8, "c2": ROLES_SMALL, "c3h": ROLES_SMALL, "c5bf16": ROLES_SMALL, "c4": ROLES_C4}


def dispatches(path):
    """[(dispatch id, kernel name, bytes)] in dispatch order."""
    out = []
    for r in csv.DictReader(open(path)):
        out.append((int(r["Dispatch_Id"]), r["Kernel_Name"], float(r["Counter_Value"]) * 1024.0))
    out.sort()
    return out


def by_role(rows, table):
    """{role: [bytes per launch, ...]} over the steps whose kernel counts match the table."""
    steps, cur = [], []
    for _, name, v in rows:
        cur.append((name, v))
        if "adam_kernel" in name:
            steps.append(cur)
            cur = []
    res = collections.defaultdict(list)
    names = {}
    for st in steps:
        for frag, roles in table:
            hits = [(n, v) for n, v in st if frag in n]
            if len(hits) != len(roles):
                continue
            for role, (n, v) in zip(roles, hits):
                res[role].append(v)
                names[role] = n
    return res, names


def keep_rows(src, dst, table):
    """The role kernels' rows of a counter CSV (the committed evidence, profiles/pmc/)."""
    frags = [f for f, _ in table] + ["adam_kernel"]
    with open(src) as fi, open(dst, "w", newline="") as fo:
        rd = csv.DictReader(fi)
        wr = csv.DictWriter(fo, fieldnames=rd.fieldnames)
        wr.writeheader()
        for r in rd:
            if any(f in r["Kernel_Name"] for f in frags):
                wr.writerow(r)


def main(fetch_csv, write_csv, out, config):
    table = ROLES.get(config, ROLES_BF16)
    tag = os.environ.get("PMC_TAG", "") or config
    for src, kind in ((fetch_csv, "fetch"), (write_csv, "write")):
        keep_rows(src, os.path.join(os.path.dirname(out), f"{tag}_{kind}.csv"), table)
    f, fn = by_role(dispatches(fetch_csv), table)
    w, _ = by_role(dispatches(write_csv), table)
    res = {}
    for role in f:
        fv, wv = f[role], w.get(role, [0.0])
        fetch, write = sum(fv) / len(fv), sum(wv) / len(wv)
        res[role] = {"kernel": fn[role], "launches": len(fv), "fetch_size_bytes_raw": fetch,
                     "write_size_bytes": write, "read_bytes_corrected": 2 * fetch,
                     "hbm_bytes_per_launch": 2 * fetch + write}
    try:
        with open(out) as fh:
            allres = json.load(fh)
    except (OSError, ValueError):
        allres = {}
    res["_source"] = {"fetch_csv": os.path.basename(fetch_csv), "write_csv": os.path.basename(write_csv),
                      "tag": tag, "keyed_by": "role (kernel + occurrence within a step, tools/pmc_summary.py)",
                      "committed_as": f"profiles/pmc/{tag}_{{fetch,write}}.csv"}
    allres[config] = res
    json.dump(allres, open(out, "w"), indent=1)
    for k, v in sorted(res.items()):
        if not k.startswith("_"):
            print(f"{k:16s} launches {v['launches']:3d}  read {v['read_bytes_corrected'] / 1e6:9.1f} MB  "
                  f"write {v['write_size_bytes'] / 1e6:9.1f} MB  ({v['kernel'][:60]})")


if __name__ == "__main__":
    main(*sys.argv[1:5])
