"""Average PMC counters per kernel from rocprofv3 --pmc csv output directories."""
import csv
import glob
import sys
from collections import defaultdict

for d in sys.argv[1:]:
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        acc = defaultdict(lambda: defaultdict(list))
        for row in csv.DictReader(open(f)):
            name = row.get("Kernel_Name", "")[:40]
            acc[name][row["Counter_Name"]].append(float(row["Counter_Value"]))
        print(f"== {f}")
        for k, cs in acc.items():
            print("  ", k, {c: round(sum(v) / len(v), 1) for c, v in cs.items()})
