"""Per-dispatch durations and inter-dispatch gaps from a rocprofv3 --kernel-trace CSV.

usage: python3 scripts/trace_gaps.py <..._kernel_trace.csv> [first] [count]
Prints one line per dispatch (index, start relative to the first, duration, gap since the previous
dispatch ended, short kernel name) for dispatches [first, first+count), then per-kernel means.
"""
import csv
import sys
from collections import defaultdict


def short(name):
    for key, s in (("widechain_kernel", "ring_chain"), ("fastchain_kernel", "fastchain"),
                   ("fastwgrad_kernel", "fastwgrad"), ("wgrad_kernel", "wgrad"), ("param_kernel", "param"),
                   ("rowchain_kernel", "rowchain")):
        if key in name:
            return s
    return name.split("(")[0][-40:]


def main():
    path = sys.argv[1]
    first = int(sys.argv[2]) if len(sys.argv) > 2 else 0
    count = int(sys.argv[3]) if len(sys.argv) > 3 else 10 ** 9
    with open(path) as f:
        rows = list(csv.DictReader(f))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    t00 = int(rows[0]["Start_Timestamp"])
    prev_end = None
    per = defaultdict(list)
    for i, r in enumerate(rows):
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        gap = None if prev_end is None else (s - prev_end) / 1e3
        if first <= i < first + count:
            print(f"{i:5d} {(s - t00) / 1e3:12.2f} us  dur {(e - s) / 1e3:8.2f}  gap {'' if gap is None else f'{gap:8.2f}'}"
                  f"  {short(r['Kernel_Name'])}")
            per[short(r["Kernel_Name"])].append((e - s) / 1e3)
        prev_end = e
    for k, v in per.items():
        print(f"{k}: n={len(v)} mean {sum(v) / len(v):.2f} us")


if __name__ == "__main__":
    main()
