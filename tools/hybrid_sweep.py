#!/usr/bin/env python3
"""Device-m05 end-to-end time vs the hybrid split (diagnostics): 256 / 1024 frames of the 4 bench
fixtures, VP8G_HOST_NS_PER_BYTE swept (larger = fewer frames on the host threads; 0 HYBRID = all
on the device), next to host-m05 mode."""
import json, os, pathlib, sys, time
ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "webp-decoder_amd"))
import vp8g
UHD = ["big/uhd_a_normal_seg4.webp", "big/uhd_b_simple_sharp3.webp", "big/uhd_c_normal_sharp6_seg1.webp", "big/uhd_d_normal_q90.webp"]
files = [(ROOT / "tests" / "fixtures" / r).read_bytes() for r in UHD]
thr = int(os.environ.get("OMP_NUM_THREADS", "16"))
vp8g.gpu_decode_webp_batch(files * 2, True, thr, device_m05=True)
for n in (256, 1024):
    batch = [files[i % 4] for i in range(n)]
    res = {"frames": n}
    vp8g.gpu_decode_webp_batch(batch, True, thr)
    res["host_m05_s"] = round(vp8g.gpu_decode_webp_batch.seconds, 3)
    for hn in (sys.argv[1:] or ["10", "20", "30", "40", "50"]):
        if hn == "off":
            os.environ["VP8G_HYBRID"] = "0"
        elif hn == "default":  # the library's own constants
            os.environ["VP8G_HYBRID"] = "1"
            os.environ.pop("VP8G_HOST_NS_PER_BYTE", None)
        else:
            os.environ["VP8G_HYBRID"] = "1"
            os.environ["VP8G_HOST_NS_PER_BYTE"] = hn
        outs, st = vp8g.gpu_decode_webp_batch(batch, True, thr, device_m05=True)
        assert all(s == 0 for s in st)
        res["device_m05_host_ns_" + hn] = round(vp8g.gpu_decode_webp_batch.seconds, 3)
        del outs
    print(json.dumps(res), flush=True)
