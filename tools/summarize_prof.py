#!/usr/bin/env python3
"""Summarise rocprofv3 csv output under a directory: per-kernel durations from
kernel traces and per-kernel counter means from PMC passes."""
import collections
import csv
import glob
import os
import sys


def short(name):
    base = name.split("(")[0]
    return base.replace("void ", "").replace("jsp::", "")


def main(root):
    for f in sorted(glob.glob(os.path.join(root, "**", "*kernel_trace.csv"), recursive=True)):
        by = collections.defaultdict(list)
        for r in csv.DictReader(open(f)):
            by[(short(r["Kernel_Name"]), r["Grid_Size_X"])].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
        print("##", os.path.relpath(f, root))
        for (k, g), v in sorted(by.items()):
            v.sort()
            print(f"  {k:40s} grid={g:>8s} n={len(v):5d} median_ns={v[len(v)//2]:8d} min_ns={v[0]:8d} "
                  f"p90_ns={v[min(len(v) - 1, len(v) * 9 // 10)]:8d} max_ns={v[-1]:8d}")
    for f in sorted(glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True)):
        agg = collections.defaultdict(lambda: collections.defaultdict(list))
        for r in csv.DictReader(open(f)):
            agg[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
        print("##", os.path.relpath(f, root))
        for k, cs in agg.items():
            if "rocclr" in k or "at::" in k:
                continue
            print(f"  {k:40s}", {c: round(sum(v) / len(v), 1) for c, v in cs.items()})


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out")
