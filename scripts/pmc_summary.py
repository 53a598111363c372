"""Average every PMC counter per pipeline kernel over its last 10 dispatches."""
import csv
import glob
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_traffic import kernel_key  # noqa: E402

d = sys.argv[1]
vals = defaultdict(lambda: defaultdict(list))
for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
    for row in csv.DictReader(open(f)):
        k = kernel_key(row.get("Kernel_Name", ""))
        if k:
            vals[k][row["Counter_Name"]].append((int(row["Dispatch_Id"]), float(row["Counter_Value"])))
for k, cs in sorted(vals.items()):
    parts = []
    for c, v in sorted(cs.items()):
        v.sort()
        last = [x for _, x in v[-10:]]
        parts.append(f"{c}={sum(last) / len(last):.4g}")
    print(k, " ".join(parts))
