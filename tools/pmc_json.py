#!/usr/bin/env python3
"""Per-MB instruction / wait / LDS summary of a tools/pmc_pass.sh run of the bench kernel, as the
committed profiles/<tag>_<kernel>_pmc.json (default kernel: quad_kernel, the bench's chain) (DESIGN.md §5 takes its numbers from it).
  tools/pmc_json.py <pmc dir> <tag> <build> [kernel filter] [workload: uhd4 | synth]"""
import collections, csv, glob, json, pathlib, sys

d, tag, build = sys.argv[1], sys.argv[2], sys.argv[3]
filt = sys.argv[4] if len(sys.argv) > 4 else "quad_kernel"
wl = sys.argv[5] if len(sys.argv) > 5 else "uhd4"
WL_TEXT = {"uhd4": "uhd4: 512 x 3840x2160, -yuvf", "synth": "synth: 512 x 3840x2160 distinct vp8_synth profile-0 frames, -yuvf"}
c = {}
kname = None
for f in sorted(glob.glob(d + "/pmc*/pmc_counter_collection.csv")):
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(f)):
        if filt in r["Kernel_Name"]:
            acc[int(r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
            kname = r["Kernel_Name"]
    if acc:
        c.update(acc[max(acc)])
mbs = 512 * 240 * 135
per_mb = {k[9:].lower() if k.startswith("SQ_INSTS_") else k.lower(): round(c[k] / mbs, 1)
          for k in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_BRANCH", "SQ_INSTS_VMEM_RD",
                    "SQ_INSTS_VMEM_WR", "SQ_INSTS_VALU_INT32") if k in c}
out = {
    "kernel": kname.split("(")[0] if kname else filt,
    "build": build,
    "workload": WL_TEXT[wl],
    "source": "rocprofv3 --pmc, one counter group per run (tools/pmc_pass.sh), last dispatch; gpurun_out/" + pathlib.Path(d).name,
    "counters": c,
    "per_mb": per_mb,
    "wave_time_shares": {
        "active_inst_any": round(c["SQ_ACTIVE_INST_ANY"] / c["SQ_WAVE_CYCLES"], 3),
        "wait_any": round(c["SQ_WAIT_ANY"] / c["SQ_WAVE_CYCLES"], 3),
        "wait_inst_any": round(c["SQ_WAIT_INST_ANY"] / c["SQ_WAVE_CYCLES"], 3),
    },
    "lds": {"bank_conflict_share": round(c["SQ_LDS_BANK_CONFLICT"] / c["SQ_LDS_IDX_ACTIVE"], 3)},
    "valu_per_simd": round(c["SQ_INSTS_VALU"] / 1024),
}
p = pathlib.Path(__file__).resolve().parents[1] / "profiles" / f"{tag}_{filt}_pmc.json"
p.write_text(json.dumps(out, indent=1) + "\n")
print(p, json.dumps(out["per_mb"]), out["wave_time_shares"], out["lds"])
