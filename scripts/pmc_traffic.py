"""Per-launch HBM-side traffic of the step's kernels from rocprofv3 --pmc passes.

Usage: python scripts/pmc_traffic.py <prof dir> <tag> <out.json> [batch dtype]

FETCH_SIZE / WRITE_SIZE are in KiB per dispatch.  On gfx950, FETCH_SIZE reports half the bytes
of wide coalesced reads (MI355X_MICROARCH.md, HBM section), so traffic = 2·FETCH + WRITE.  Both
counters come from separate passes (they cannot share one).  Averages are over every dispatch
of the kernel in the profiled bench run.
"""
import csv
import glob
import json
import sys
from collections import defaultdict


def short(name):
    if any(k in name for k in ("rowchain_kernel", "fastchain_kernel", "widechain_kernel", "f32chain_kernel")):
        return "rowchain"
    if "wgrad_kernel" in name:  # wgrad_kernel and fastwgrad_kernel
        return "wgrad_adam"
    if "param_kernel" in name:
        return "param"
    return None


def main():
    d, tag, out = sys.argv[1], sys.argv[2], sys.argv[3]
    batch = int(sys.argv[4]) if len(sys.argv) > 4 else 1024
    dtype = sys.argv[5] if len(sys.argv) > 5 else "bf16"
    vals = defaultdict(lambda: defaultdict(list))
    for f in sorted(glob.glob(f"{d}/**/{tag}_pmc*counter_collection.csv", recursive=True)):
        for row in csv.DictReader(open(f)):
            k = short(row.get("Kernel_Name", ""))
            if k and row["Counter_Name"] in ("FETCH_SIZE", "WRITE_SIZE"):
                vals[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
    res = {"source": f"rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes, tag {tag}",
           "correction": "traffic = 2*FETCH_SIZE + WRITE_SIZE (gfx950 FETCH_SIZE counts half of wide reads)",
           "config": {"batch": batch, "dtype": dtype}, "kernels": {}}
    for k, cs in vals.items():
        fetch = sum(cs["FETCH_SIZE"]) / max(len(cs["FETCH_SIZE"]), 1) * 1024
        write = sum(cs["WRITE_SIZE"]) / max(len(cs["WRITE_SIZE"]), 1) * 1024
        res["kernels"][k] = {"fetch_bytes_raw": round(fetch), "write_bytes": round(write),
                             "traffic_bytes": round(2 * fetch + write),
                             "dispatches": len(cs["FETCH_SIZE"])}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
