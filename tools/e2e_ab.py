#!/usr/bin/env python3
"""Interleaved A/B of the end-to-end device-m05 leg (bench `end_to_end.device_m05_large`) between
libvp8g builds (diagnostics; verdict r04 #4).

The leg loads one libvp8g per process (vp8g.py reads VP8G_LIB), so every (library, repeat) is its
own child process, run in the order lib1, lib2, ..., lib1, lib2, ...; each child prints the seconds
of its calls and whether every frame matched the reference's sha256.  With --trace the first run
of each library also writes the pipeline's chunk trace (VP8G_PIPE_TRACE=1) next to the output.

  python tools/e2e_ab.py [--frames 1024] [--reps 3] [--trace DIR] lib1.so lib2.so ...
"""
import argparse
import json
import os
import pathlib
import subprocess
import sys

ROOT = pathlib.Path(__file__).resolve().parents[1]


def child(frames: int, calls: int) -> None:
    sys.path.insert(0, str(ROOT))
    sys.path.insert(0, str(ROOT / "webp-decoder_amd"))
    import hashlib
    import bench
    import vp8g
    manifest = json.loads((ROOT / "tests" / "golden" / "manifest.json").read_text())
    files = [(ROOT / "tests" / "fixtures" / r).read_bytes() for r in bench.UHD]
    batch = [files[i % 4] for i in range(frames)]
    threads = bench.cpu_share()
    vp8g.gpu_decode_webp_batch(batch[:8], True, threads, device_m05=True)  # warm
    secs, ok = [], True
    for _ in range(calls):
        outs, st = vp8g.gpu_decode_webp_batch(batch, True, threads, device_m05=True)
        secs.append(round(vp8g.gpu_decode_webp_batch.seconds, 4))
        ok = ok and all(s == 0 for s in st) and all(
            hashlib.sha256(outs[i]).hexdigest() == manifest["files"][bench.UHD[i % 4]]["yuvf_sha256"]
            for i in range(0, frames, 16))
        del outs
    print(json.dumps({"seconds": secs, "threads": threads, "parity_sampled": ok}), flush=True)


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=1024)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--calls", type=int, default=2)
    ap.add_argument("--trace", default="")
    ap.add_argument("--child", action="store_true")
    ap.add_argument("libs", nargs="*")
    a = ap.parse_args()
    if a.child:
        child(a.frames, a.calls)
        return
    res = {lib: [] for lib in a.libs}
    for rep in range(a.reps):
        for i, lib in enumerate(a.libs):
            env = dict(os.environ, VP8G_LIB=str(pathlib.Path(lib).resolve()))
            log = None
            if a.trace and rep == 0:
                env["VP8G_PIPE_TRACE"] = "1"
                log = pathlib.Path(a.trace) / f"trace_{i}.log"
            p = subprocess.run([sys.executable, __file__, "--child", "--frames", str(a.frames), "--calls", str(a.calls)],
                               env=env, capture_output=True, text=True, timeout=600)
            if log:
                log.write_text(p.stderr)
            if p.returncode != 0:
                print(p.stderr[-2000:], file=sys.stderr)
                sys.exit(f"{lib}: child failed rc={p.returncode}")
            d = json.loads(p.stdout.strip().splitlines()[-1])
            res[lib].append(d)
            print(json.dumps({"lib": lib, "rep": rep, **d}), flush=True)
    for lib, runs in res.items():
        s = sorted(x for r in runs for x in r["seconds"])
        med = s[len(s) // 2]
        print(json.dumps({"lib": lib, "median_s": med, "mp_per_s": round(a.frames * 3840 * 2160 / 1e6 / med, 1),
                          "all_s": s, "parity": all(r["parity_sampled"] for r in runs)}), flush=True)


if __name__ == "__main__":
    main()
