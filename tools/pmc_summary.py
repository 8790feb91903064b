#!/usr/bin/env python3
"""Per-kernel PMC summary of a tools/pmc_pass.sh / pmc_enc.sh output directory (last dispatch of
each kernel whose name contains the filter).  Usage: tools/pmc_summary.py <dir> <name filter>"""
import collections, csv, glob, sys
d, filt = sys.argv[1], sys.argv[2]
for f in sorted(glob.glob(d + "/pmc*/pmc_counter_collection.csv")):
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(f)):
        if filt in r["Kernel_Name"]:
            acc[int(r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
    if acc:
        last = acc[max(acc)]
        print(f.split("/")[-2], len(acc), {k: "%.4g" % v for k, v in sorted(last.items())})
