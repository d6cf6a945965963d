"""Average rocprofv3 PMC counters per kernel (dispatch-averaged) across group directories."""
import collections
import csv
import glob
import sys

agg = collections.defaultdict(lambda: collections.defaultdict(float))
cnt = collections.defaultdict(set)
for g in sorted(glob.glob(sys.argv[1] + "/g*/pmc_counter_collection.csv")):
    for r in csv.DictReader(open(g)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "")[-48:]
        if len(sys.argv) > 2 and sys.argv[2] not in k:
            continue
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        cnt[(k, r["Counter_Name"])].add(r["Dispatch_Id"])
for k, v in agg.items():
    print(k)
    for c, x in sorted(v.items()):
        print(f"   {c:36s} {x / max(1, len(cnt[(k, c)])):.4e}")
