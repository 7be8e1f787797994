"""Per-kernel mean of every PMC counter in a rocprofv3 counter-collection directory, for kernels matching a filter:
    python tools/pmc_kernel_summary.py DIR FILTER"""
import collections
import csv
import glob
import sys

d, filt = sys.argv[1], sys.argv[2]
files = glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in files:
    for r in csv.DictReader(open(f)):
        name = r.get("Kernel_Name", "")
        if filt not in name:
            continue
        acc[name[:70]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, ctrs in acc.items():
    print(k, " ".join(f"{c}={sum(v) / len(v):.4g}" for c, v in sorted(ctrs.items())))
