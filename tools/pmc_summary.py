"""Summarise rocprofv3 --pmc CSVs per kernel (averaged over dispatches)."""
import csv, glob, sys, collections
root = sys.argv[1]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(f"{root}/p*/run_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        short = k.split("(")[0].replace("void ", "").replace("rs2::", "").replace("(anonymous namespace)::", "")
        acc[short][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in acc.items():
    if "at::" in k or "rocclr" in k:
        continue
    print(k)
    for c, v in sorted(cs.items()):
        print(f"   {c:28s} mean={sum(v)/len(v):16.1f}  n={len(v)}")
