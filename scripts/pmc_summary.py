"""Summarise rocprofv3 PMC csv files: per kernel, mean of each counter per dispatch."""
import csv
import glob
import sys
from collections import defaultdict

d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof"
tag = sys.argv[2] if len(sys.argv) > 2 else "r01"
acc = defaultdict(lambda: defaultdict(list))
for f in sorted(glob.glob(f"{d}/**/{tag}_pmc*counter_collection.csv", recursive=True)):
    for row in csv.DictReader(open(f)):
        k = row.get("Kernel_Name", "?")
        k = k.split("(")[0][:60]
        acc[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
for k, cs in acc.items():
    print(k)
    for c, v in sorted(cs.items()):
        print(f"   {c:28s} {sum(v) / len(v):16.1f}  (n={len(v)})")
