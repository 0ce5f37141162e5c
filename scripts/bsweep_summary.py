"""Summarise scripts/bsweep.sh: per B_local, bench throughput and per-kernel MFMA utilisation.

whole-GPU MFMA utilisation = SQ_VALU_MFMA_BUSY_CYCLES / (kernel cycles x 1024 SIMDs), with the
kernel cycles = the un-profiled kernel time (bench kernels_ms) x 2.4 GHz (peak engine clock: an
upper bound on the cycles, so a lower bound on the utilisation).  per-active-CU = the same over
the CUs that hold a workgroup: min(256, workgroups) (row chain: B/16 workgroups; dW: 281).
(Round 2 printed GRBM_GUI_ACTIVE / 8 / kernel time as a "clock" column; it read 3.9-5.8 GHz on a
2.4 GHz part because under --pmc the counter spans the profiled dispatch with its serialisation
overhead, not the kernel's un-profiled time — it measured nothing useful and is gone.)
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/bsweep"
rows = []
for f in sorted(glob.glob(f"{d}/bench_*.json"), key=lambda p: int(p.rsplit("_", 1)[1].split(".")[0])):
    B = int(f.rsplit("_", 1)[1].split(".")[0])
    b = json.load(open(f))
    acc = defaultdict(lambda: defaultdict(list))
    for c in glob.glob(f"{d}/**/pmc_{B}*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(c)):
            k = r.get("Kernel_Name", "?")
            k = "rowchain" if ("fastchain" in k or "widechain" in k) else "wgrad_adam" if "fastwgrad" in k else None
            if k:
                acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    rows.append((B, b, {k: {c: sum(v) / len(v) for c, v in cs.items()} for k, cs in acc.items()}))

print("| B_local | traj/s | µs/step | row chain µs | dW+Adam µs | step TFLOP/s | kernel | MFMA insts | MFMA busy (whole GPU) | MFMA busy (active CUs) |")
print("|---|---|---|---|---|---|---|---|---|---|")
for B, b, pm in rows:
    km = b["roofline"]["kernels_ms"]
    tfs = b["value"] * b["flop_per_traj"] / 1e12
    for k in ("rowchain", "wgrad_adam"):
        c = pm.get(k, {})
        busy, gui = c.get("SQ_VALU_MFMA_BUSY_CYCLES"), c.get("GRBM_GUI_ACTIVE")
        wg = B // 16 if k == "rowchain" else 281
        if busy is not None and gui:
            cyc = km[k] * 1e-3 * 2.4e9
            whole = busy / (cyc * 1024)
            act = whole * 256 / min(256, wg)
            u = f"{100 * whole:.2f} % | {100 * act:.2f} %"
        else:
            u = "— | —"
        head = (f"| {B} | {b['value'] / 1e6:.1f} M | {b['ms_per_step'] * 1e3:.1f} | {km['rowchain'] * 1e3:.1f} | "
                f"{km['wgrad_adam'] * 1e3:.1f} | {tfs:.0f} |" if k == "rowchain" else "| | | | | | |")
        print(f"{head} {k} | {c.get('SQ_INSTS_MFMA', float('nan')):.0f} | {u} |")
