#!/usr/bin/env python3
"""Fold the summary lines of in-process A/B runs (gpurun_out/ab_<tag>/<workload>.jsonl, written by
tools/gpu_round.sh ab) into one committed JSON file under profiles/.

Usage: tools/fold_ab.py out.json tag=description [tag=description ...]   (merges into out.json)
"""
import json, os, sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
out, pairs = sys.argv[1], sys.argv[2:]
res = json.load(open(out)) if os.path.exists(out) else {}  # (tags already folded are kept or replaced)
for p in pairs:
    tag, _, what = p.partition("=")
    d = os.path.join(ROOT, "gpurun_out", "ab_" + tag)
    runs = {}
    for f in sorted(os.listdir(d)):
        if not f.endswith(".jsonl"):
            continue
        rows = []
        for line in open(os.path.join(d, f)):
            try:
                r = json.loads(line)
            except ValueError:
                continue
            if "median_ms" in r:
                rows.append({k: r[k] for k in ("lib", "median_ms", "min_ms", "parity", "digests_sha") if k in r})
        runs[f[:-6]] = rows
    res[tag] = {"what": what, "workloads": runs}
json.dump(res, open(out, "w"), indent=1)
print(out, len(res), "A/B runs")
