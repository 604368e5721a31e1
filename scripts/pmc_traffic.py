"""Per-launch HBM traffic of the bench line's sampler kernels from two rocprofv3 --pmc passes (FETCH_SIZE and
WRITE_SIZE cannot share a pass on gfx950), corrected as MI355X_MICROARCH.md §HBM prescribes: FETCH_SIZE (KiB)
doubled (gfx950 tallies the 128-B requests of wide coalesced reads -- 16-B-per-lane loads and LDS-DMA alike
-- at 64 B), WRITE_SIZE (KiB) as is. Writes profiles/pmc_traffic.json: {kernel family: bytes per launch}.
    python scripts/pmc_traffic.py <fetch-pass dir> <write-pass dir> [out.json]"""
import csv
import glob
import json
import statistics
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
    # the median over the pass's launches: the first launch of a fresh process can read several times more (cold
    # first touch of the output and scratch pages: 97 MB against 5 MB on one box), which is not the steady state
    return {k: float(statistics.median(v.values())) for k, v in vals.items() if v}, \
        {k: max(v.values()) for k, v in vals.items() if v}


def main():
    (fetch, fetch_max), (write, write_max) = per_launch(sys.argv[1], "FETCH_SIZE"), per_launch(sys.argv[2], "WRITE_SIZE")
    out = {"source": [sys.argv[1], sys.argv[2]],
           "correction": "bytes = (2 FETCH_SIZE + WRITE_SIZE) KiB (MI355X_MICROARCH.md HBM: gfx950 FETCH_SIZE = 1/2 of wide reads)",
           "statistic": "median over the pass's launches (max = the cold first launch, listed beside)"}
    for k in fetch:
        out[k] = {"fetch_kib": fetch[k], "write_kib": write.get(k), "hbm_bytes_per_launch":
                  (2.0 * fetch[k] + write.get(k, 0.0)) * 1024.0,
                  "max_launch_fetch_kib": fetch_max[k], "max_launch_write_kib": write_max.get(k)}
    path = sys.argv[3] if len(sys.argv) > 3 else "profiles/pmc_traffic.json"
    json.dump(out, open(path, "w"), indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
