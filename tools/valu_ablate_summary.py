#!/usr/bin/env python3
"""Summarise tools/valu_ablate.sh: per-variant SQ_INSTS_* per frame_kernel dispatch.
Usage: tools/valu_ablate_summary.py <outdir>"""
import csv, glob, sys, collections
out = sys.argv[1]
for v in ["base", "abl1", "abl2", "abl4", "abl8"]:
    fs = glob.glob(f"{out}/{v}/**/*counter_collection.csv", recursive=True)
    if not fs:
        continue
    tot, disp = collections.defaultdict(float), set()
    for r in csv.DictReader(open(fs[0])):
        if "frame_kernel" in r["Kernel_Name"]:
            tot[r["Counter_Name"]] += float(r["Counter_Value"])
            disp.add(r["Dispatch_Id"])
    n = len(disp)
    print(v, {k: round(x / n / 1e6, 1) for k, x in sorted(tot.items())}, "M per dispatch")
