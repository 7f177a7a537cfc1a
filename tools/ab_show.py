"""Print tools/gpu_ab.sh results: env-steps/s per (workload, library), both repetitions."""
import glob
import json
import os
import sys
from collections import defaultdict

d = sys.argv[1]
res = defaultdict(list)
for f in sorted(glob.glob(os.path.join(d, "*.json"))):
    b = os.path.basename(f)[:-5]
    w, rest = b.split("_", 1)
    n, rep = rest.rsplit("_", 1)
    try:
        j = json.loads(open(f).read().strip().splitlines()[-1])
        res[(w, n)].append((j["value"], j["roofline"]["k1_ms"]))
    except Exception as e:  # noqa: BLE001
        res[(w, n)].append((None, str(e)))
for (w, n), v in sorted(res.items()):
    print(f"{w:8s} {n:40s} " + "  ".join(f"{a} ({b} ms)" for a, b in v))
