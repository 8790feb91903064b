#!/usr/bin/env python3
"""Host-to-host rate of the drop-in host API (vp8g_reconstruct_batch: H2D of the decoded
arrays, one fused launch, D2H into yuv420_alloc()ed planes) on a batch of 4K frames.
This is the PCIe-inclusive figure DESIGN.md quotes next to the device-resident bench value;
it is never the bench `value`.  Usage: python tools/pcie_rate.py [frames] [reps]"""
import ctypes as C
import json
import pathlib
import sys
import time

ROOT = pathlib.Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "webp-decoder_amd"))
import vp8g  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 32
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
fx = ["big/uhd_a_normal_seg4.webp", "big/uhd_b_simple_sharp3.webp", "big/uhd_c_normal_sharp6_seg1.webp",
      "big/uhd_d_normal_q90.webp"]
src = [vp8g.decode_file(ROOT / "tests" / "fixtures" / f) for f in fx]
frames = [src[i % 4] for i in range(n)]
lib = vp8g.gpu_lib()
kfs = (C.POINTER(vp8g.Vp8KeyFrameHeader) * n)(*[C.pointer(f.kf) for f in frames])
frs = (C.POINTER(vp8g.Vp8DecodedFrame) * n)(*[C.pointer(f.frame) for f in frames])
best = None
for r in range(reps + 1):
    imgs = (vp8g.Yuv420Image * n)()
    t0 = time.perf_counter()
    rc = lib.vp8g_reconstruct_batch(C.cast(kfs, C.c_void_p), C.cast(frs, C.c_void_p), n, 1, imgs)
    dt = time.perf_counter() - t0
    if rc != 0:
        raise SystemExit(f"batch failed: {lib.vp8g_last_error()!r}")
    for i in range(n):
        lib.yuv420_free(C.byref(imgs[i]))
    if r > 0:
        best = dt if best is None else min(best, dt)
mp = n * 3840 * 2160 / 1e6
in_bytes = n * src[0].mb_total * 820
print(json.dumps({"api": "vp8g_reconstruct_batch (host buffers, pageable)", "frames": n, "seconds": round(best, 4),
                  "mp_per_s": round(mp / best, 1), "h2d_bytes": in_bytes,
                  "d2h_bytes": n * vp8g.i420_size(3840, 2160)}))
