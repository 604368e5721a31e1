"""Summarise rocprofv3 --pmc CSVs (gpurun_out/<tag>/pmc_*/pmc_counter_collection.csv) for one kernel
and derive the per-launch HBM traffic the way MI355X_MICROARCH.md §HBM prescribes:
FETCH_SIZE / WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE reports half the bytes of wide coalesced
reads (doubled here; our HBM reads are the 1 KiB-per-wave LDS-DMA weight pieces and dwordx4
prologue loads), WRITE_SIZE is taken as is (the output stores are dword stores -- uncalibrated,
see DESIGN.md).
   python scripts/pmc_summary.py <tag> [kernel-substring] [--json out.json]"""
import csv
import glob
import json
import sys
from collections import defaultdict


def summarise(tag, match="em_sampler"):
    vals = defaultdict(list)
    durs = []
    for f in sorted(glob.glob(f"gpurun_out/{tag}/pmc_*/pmc_counter_collection.csv") +
                    glob.glob(f"gpurun_out/{tag}/pmc_counter_collection.csv")):
        seen = {}
        for row in csv.DictReader(open(f)):
            if match not in row["Kernel_Name"]:
                continue
            key = (row["Dispatch_Id"], row["Counter_Name"])
            seen[key] = seen.get(key, 0.0) + float(row["Counter_Value"])
            durs.append(int(row["End_Timestamp"]) - int(row["Start_Timestamp"]))
        for (d, c), v in seen.items():
            vals[c].append(v)
    out = {c: sum(v) / len(v) for c, v in vals.items()}
    out["dispatch_ns_mean"] = sum(durs) / len(durs) if durs else None
    if "FETCH_SIZE" in out and "WRITE_SIZE" in out:
        out["hbm_bytes_per_launch"] = (2.0 * out["FETCH_SIZE"] + out["WRITE_SIZE"]) * 1024.0
    if "GRBM_GUI_ACTIVE" in out and out["dispatch_ns_mean"]:
        out["effective_clock_GHz"] = out["GRBM_GUI_ACTIVE"] / 8.0 / out["dispatch_ns_mean"]
    return out


if __name__ == "__main__":
    tag = sys.argv[1]
    match = sys.argv[2] if len(sys.argv) > 2 and not sys.argv[2].startswith("--") else "em_sampler"
    res = summarise(tag, match)
    for k, v in sorted(res.items()):
        print(f"{k:28s} {v}")
    if "--json" in sys.argv:
        path = sys.argv[sys.argv.index("--json") + 1]
        json.dump({"source": f"gpurun_out/{tag}", "kernel_match": match, **res}, open(path, "w"), indent=1)
