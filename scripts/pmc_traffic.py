"""Per-launch HBM traffic of the bench line's sampler kernels from two rocprofv3 --pmc passes (FETCH_SIZE and
WRITE_SIZE cannot share a pass on gfx950), corrected as MI355X_MICROARCH.md §HBM prescribes: FETCH_SIZE (KiB)
doubled (gfx950 tallies the 128-B requests of wide coalesced reads -- 16-B-per-lane loads and LDS-DMA alike
-- at 64 B), WRITE_SIZE (KiB) as is. Writes profiles/pmc_traffic.json: {kernel family: bytes per launch}.
    python scripts/pmc_traffic.py <fetch-pass dir> <write-pass dir> [out.json]"""
import csv
import glob
import json
import sys
from collections import defaultdict

FAMILIES = ("x3k_sampler_kernel", "x3_sampler_kernel", "em_sampler_kernel", "f32_sampler_kernel")


def per_launch(d, counter):
    vals = defaultdict(lambda: defaultdict(float))
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for row in csv.DictReader(open(f)):
            if row["Counter_Name"] != counter:
                continue
            fam = next((k for k in FAMILIES if k in row["Kernel_Name"] and
                        not (k == "x3_sampler_kernel" and "x3k_sampler_kernel" in row["Kernel_Name"])), None)
            if fam:
                vals[fam][row["Dispatch_Id"]] += float(row["Counter_Value"])
    return {k: sum(v.values()) / len(v) for k, v in vals.items() if v}


def main():
    fetch, write = per_launch(sys.argv[1], "FETCH_SIZE"), per_launch(sys.argv[2], "WRITE_SIZE")
    out = {"source": [sys.argv[1], sys.argv[2]],
           "correction": "bytes = (2 FETCH_SIZE + WRITE_SIZE) KiB (MI355X_MICROARCH.md HBM: gfx950 FETCH_SIZE = 1/2 of wide reads)"}
    for k in fetch:
        out[k] = {"fetch_kib": fetch[k], "write_kib": write.get(k), "hbm_bytes_per_launch":
                  (2.0 * fetch[k] + write.get(k, 0.0)) * 1024.0}
    path = sys.argv[3] if len(sys.argv) > 3 else "profiles/pmc_traffic.json"
    json.dump(out, open(path, "w"), indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
