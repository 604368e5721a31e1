"""Summarise rocprofv3 --pmc CSVs (gpurun_out/<tag>/pmc_*/pmc_counter_collection.csv) per kernel."""
import csv
import glob
import sys
from collections import defaultdict

tag = sys.argv[1] if len(sys.argv) > 1 else "pmc"
match = sys.argv[2] if len(sys.argv) > 2 else "em_sampler"
vals = defaultdict(list)
durs = []
for f in sorted(glob.glob(f"gpurun_out/{tag}/pmc_*/pmc_counter_collection.csv")):
    seen = {}
    for row in csv.DictReader(open(f)):
        if match not in row["Kernel_Name"]:
            continue
        key = (row["Dispatch_Id"], row["Counter_Name"])
        seen[key] = seen.get(key, 0.0) + float(row["Counter_Value"])
        durs.append(int(row["End_Timestamp"]) - int(row["Start_Timestamp"]))
    for (d, c), v in seen.items():
        vals[c].append(v)
for c, v in sorted(vals.items()):
    print(f"{c:28s} {sum(v)/len(v):16.4g}   (n={len(v)})")
if durs:
    print("mean dispatch ns", sum(durs) / len(durs))
