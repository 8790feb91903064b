#!/usr/bin/env python3
"""Host-m05 end-to-end time vs frames per chunk (VP8G_CHUNK_FRAMES, diagnostics), 256 and 1024 x 4K."""
import os, pathlib, sys, json
ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "webp-decoder_amd"))
import vp8g
UHD = ["big/uhd_a_normal_seg4.webp", "big/uhd_b_simple_sharp3.webp", "big/uhd_c_normal_sharp6_seg1.webp", "big/uhd_d_normal_q90.webp"]
files = [(ROOT / "tests" / "fixtures" / r).read_bytes() for r in UHD]
thr = 16
vp8g.gpu_decode_webp_batch(files * 2, True, thr)
res = {}
for rnd in range(3):
    for n in (256, 1024):
        batch = [files[i % 4] for i in range(n)]
        for cf in ("16", "32", "64"):
            os.environ["VP8G_CHUNK_FRAMES"] = cf
            outs, st = vp8g.gpu_decode_webp_batch(batch, True, thr)
            assert all(s == 0 for s in st); del outs
            res.setdefault(f"host_{n}_{cf}", []).append(round(vp8g.gpu_decode_webp_batch.seconds, 3))
print(json.dumps(res))
