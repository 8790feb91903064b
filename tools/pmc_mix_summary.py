#!/usr/bin/env python3
"""Summarise a tools/pmc_mix.sh run: per library, the bench kernel's SQ counters per launch and per
macroblock (512 x 4K = 16 588 800 MBs), averaged over its frame_kernel dispatches (diagnostics).

  python tools/pmc_mix_summary.py gpurun_out/pmc_<tag> [out.json]
"""
import csv
import glob
import json
import pathlib
import sys

src = pathlib.Path(sys.argv[1])
libs = [l.split(None, 1) for l in (src / "libs.txt").read_text().splitlines() if l.strip()]
MBS = 512 * 240 * 135
res = {}
for i, lib in libs:
    f = glob.glob(str(src / f"mix{i}" / "**" / "*counter_collection.csv"), recursive=True)[0]
    tot, disp = {}, {}
    for r in csv.DictReader(open(f)):
        if "frame_kernel" not in r["Kernel_Name"] and "quad_kernel" not in r["Kernel_Name"]:
            continue
        c = r["Counter_Name"]
        tot[c] = tot.get(c, 0.0) + float(r["Counter_Value"])
        disp.setdefault(c, set()).add(r["Dispatch_Id"])
    per = {c: tot[c] / len(disp[c]) for c in tot}
    wc = per.get("SQ_WAVE_CYCLES", 0.0) or 1.0
    res[lib] = {
        "dispatches": len(next(iter(disp.values()))) if disp else 0,
        "per_mb": {c.replace("SQ_INSTS_", "").lower(): round(per[c] / MBS, 1) for c in per if c.startswith("SQ_INSTS_")},
        "wave_time_shares": {c.replace("SQ_", "").lower(): round(per[c] / wc, 3)
                             for c in ("SQ_ACTIVE_INST_ANY", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY") if c in per},
        "wave_quad_cycles_per_launch": round(wc),
    }
out = json.dumps(res, indent=1)
print(out)
if len(sys.argv) > 2:
    pathlib.Path(sys.argv[2]).write_text(out + "\n")
