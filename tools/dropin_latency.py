#!/usr/bin/env python3
"""Per-call wall time of the drop-in entry point vp8_reconstruct_keyframe_yuv_filtered (host
Vp8DecodedFrame in, malloc'ed I420 out: H2D, one launch, D2H), as the reference CLI calls it,
for one 4K and one 1080p fixture.  Usage: python tools/dropin_latency.py [reps]"""
import ctypes as C
import json
import pathlib
import sys
import time

ROOT = pathlib.Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "webp-decoder_amd"))
import vp8g  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
lib = vp8g.gpu_lib()
res = {}
for name in ["big/uhd_a_normal_seg4.webp", "big/fhd_normal_sharp5.webp"]:
    p = ROOT / "tests" / "fixtures" / name
    if not p.exists():
        continue
    f = vp8g.decode_file(p)
    ts = []
    for r in range(reps + 1):
        img = vp8g.Yuv420Image()
        t0 = time.perf_counter()
        rc = lib.vp8_reconstruct_keyframe_yuv_filtered(C.byref(f.kf), C.byref(f.frame), C.byref(img))
        dt = time.perf_counter() - t0
        if rc != 0:
            raise SystemExit(f"call failed: {lib.vp8g_last_error()!r}")
        lib.yuv420_free(C.byref(img))
        if r > 0:
            ts.append(dt)
    ts.sort()
    res[name] = {"w": f.width, "h": f.height, "median_ms": round(1e3 * ts[len(ts) // 2], 3),
                 "min_ms": round(1e3 * ts[0], 3)}
print(json.dumps(res))
