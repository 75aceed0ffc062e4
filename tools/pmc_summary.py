"""Sum rocprofv3 counter_collection.csv rows per (kernel, counter) -> JSON (dev tool)."""
import csv
import json
import sys
from collections import defaultdict

# --all keeps every kernel (calibration runs); default: the library's kernels only
ALL = "--all" in sys.argv[1:]
paths = [a for a in sys.argv[1:] if a != "--all"]
tot = defaultdict(lambda: defaultdict(float))
disp = defaultdict(set)
for path in paths:
    for r in csv.DictReader(open(path)):
        k = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0]
        tot[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[k].add((path, r["Dispatch_Id"]))
out = {}
for k, c in tot.items():
    if not ALL and "cordahip" not in k:
        continue
    out[k] = dict(c)
    out[k]["dispatches_per_pass"] = len(disp[k]) / max(1, len(paths))
print(json.dumps(out, indent=1))
