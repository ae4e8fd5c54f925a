#!/usr/bin/env python3
"""Average each counter over the dispatches of one kernel across all
rocprofv3 --pmc pass directories under <dir>."""
import csv
import glob
import sys
from collections import defaultdict

root, kernel = sys.argv[1], sys.argv[2]
acc = defaultdict(lambda: defaultdict(float))
for path in glob.glob(f"{root}/p*/**/*counter_collection.csv", recursive=True):
    with open(path) as f:
        for row in csv.DictReader(f):
            if kernel in row.get("Kernel_Name", ""):
                acc[row["Counter_Name"]][row["Dispatch_Id"]] += float(row["Counter_Value"])
for name in sorted(acc):
    v = list(acc[name].values())
    print(f"{name:28s} {sum(v) / len(v):16.1f}  (n={len(v)})")
