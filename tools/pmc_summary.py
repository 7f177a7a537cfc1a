"""Summarise rocprofv3 PMC passes (tools/gpu_pmc.sh) per kernel: per-dispatch averages."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def load(dirpath):
    agg = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(dirpath, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            # "pk_render_kernel(...)", "void pk_step_kernel<true>(...)" -> the kernel's base name
            k = row.get("Kernel_Name", "?").split("(")[0].split("<")[0].split(" ")[-1]
            agg[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
    return agg


if __name__ == "__main__":
    d = sys.argv[1]
    agg = load(d)
    out = {}
    for k, cs in agg.items():
        out[k] = {c: sum(v) / len(v) for c, v in cs.items()}   # mean per dispatch
    print(json.dumps(out, indent=1))
