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

# Concurrent callers (verdict r02 #7): calls per second of the drop-in entry point from 1, 2, 4 and 8
# threads (each call leases one of the library's eight device contexts, its own stream and buffers).
import concurrent.futures as cf  # noqa: E402

conc = {}
for name in ["big/uhd_a_normal_seg4.webp", "big/fhd_normal_sharp5.webp"]:
    p = ROOT / "tests" / "fixtures" / name
    if not p.exists():
        continue
    f = vp8g.decode_file(p)

    def one(_):
        img = vp8g.Yuv420Image()
        rc = lib.vp8_reconstruct_keyframe_yuv_filtered(C.byref(f.kf), C.byref(f.frame), C.byref(img))
        if rc != 0:
            raise RuntimeError(lib.vp8g_last_error())
        lib.yuv420_free(C.byref(img))

    per = {}
    for th in (1, 2, 4, 8):
        calls = 8 * reps
        with cf.ThreadPoolExecutor(th) as ex:
            list(ex.map(one, range(th)))  # (warm every context)
            t0 = time.perf_counter()
            list(ex.map(one, range(calls)))
            dt = time.perf_counter() - t0
        per[th] = {"calls": calls, "seconds": round(dt, 3), "calls_per_s": round(calls / dt, 1),
                   "MP_per_s": round(calls * f.width * f.height / dt / 1e6, 1)}
    conc[name] = per
print(json.dumps({"concurrent": conc}))
