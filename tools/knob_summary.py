"""Summarise gpu_knob.sh logs: ms/step per setting and round.  python tools/knob_summary.py <dir>"""
import glob
import json
import os
import sys

d = sys.argv[1]
for name in sorted(glob.glob(os.path.join(d, "*.name")), key=lambda p: int(os.path.basename(p).split(".")[0])):
    i = os.path.basename(name).split(".")[0]
    vals = []
    for log in sorted(glob.glob(os.path.join(d, f"{i}_*.log"))):
        for line in open(log):
            if line.startswith("{"):
                vals.append(json.loads(line)["ms_per_step"])
    print(f"{open(name).read().strip():40s} " + " ".join(f"{v:.3f}" for v in vals))
