#!/usr/bin/env python3
"""Per-call H2D / kernel / D2H split of the drop-in entry point from a tools/dropin_profile.sh run
(rocprofv3 kernel + memory-copy traces of tools/dropin_latency.py), as profiles/<tag>_dropin.json.
  tools/dropin_summary.py <tag>"""
import csv, json, pathlib, statistics, sys

tag = sys.argv[1]
ROOT = pathlib.Path(__file__).resolve().parents[1]
d = ROOT / "gpurun_out" / f"dropin_{tag}"
ev = []
for r in csv.DictReader(open(d / "trace" / "trace_memory_copy_trace.csv")):
    ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "h2d" if "HOST_TO_DEVICE" in r["Direction"] else "d2h"))
for r in csv.DictReader(open(d / "trace" / "trace_kernel_trace.csv")):
    kn = r["Kernel_Name"]
    ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "kernel:" + (kn[:kn.index(">") + 1] if "frame_kernel" in kn else kn.split("(")[0])))
ev.sort()
# a call = the events from one frame_kernel's preceding H2D burst to its D2H burst
calls, cur = [], []
for e in ev:
    if e[2] == "h2d" and cur and any(x[2] == "d2h" for x in cur):
        calls.append(cur)
        cur = []
    cur.append(e)
if cur:
    calls.append(cur)
lat = json.loads((d / "latency.json").read_text())
names = list(lat)
per = len(calls) // len(names)
out = {"source": f"gpurun_out/dropin_{tag} (rocprofv3 --kernel-trace --memory-copy-trace of tools/dropin_latency.py; the first call per fixture, which allocates, is dropped)", "calls": {}}
for i, n in enumerate(names):
    cs = calls[i * per + 1:(i + 1) * per]
    def med(f):
        return round(statistics.median(f(c) for c in cs) / 1e6, 3)
    out["calls"][n] = {
        "wall_ms_median": lat[n]["median_ms"],
        "h2d_ms": med(lambda c: sum(e[1] - e[0] for e in c if e[2] == "h2d")),
        "kernels_ms": med(lambda c: sum(e[1] - e[0] for e in c if e[2].startswith("kernel"))),
        "recon_kernel_ms": med(lambda c: sum(e[1] - e[0] for e in c if "frame_kernel" in e[2])),
        "d2h_ms": med(lambda c: sum(e[1] - e[0] for e in c if e[2] == "d2h")),
        "span_ms": med(lambda c: c[-1][1] - c[0][0]),
        "copies": statistics.median(sum(1 for e in c if e[2] in ("h2d", "d2h")) for c in cs),
        "kernel_names": sorted({e[2][7:] for e in cs[0] if e[2].startswith("kernel")}),
    }
p = ROOT / "profiles" / f"{tag}_dropin.json"
p.write_text(json.dumps(out, indent=1) + "\n")
print(json.dumps(out, indent=1))
