"""Wall clock of the end-to-end batch path, host m05 vs device m05, on the 4 bench fixtures
(3840x2160) round-robin.  Usage: python tools/m05_probe.py N [threads]"""
import hashlib
import json
import pathlib
import sys
import time

import torch  # noqa: F401  (HIP runtime first, as bench.py)

ROOT = pathlib.Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "webp-decoder_amd"))
sys.path.insert(0, str(ROOT))
import vp8g  # noqa: E402
from bench import FIXTURES  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 256
threads = int(sys.argv[2]) if len(sys.argv) > 2 else 16
man = json.loads((ROOT / "tests" / "golden" / "manifest.json").read_text())
files = [(ROOT / "tests" / "fixtures" / r).read_bytes() for r in FIXTURES]
batch = [files[i % 4] for i in range(n)]
for dev in (True, False):
    vp8g.gpu_decode_webp_batch(batch[:8], True, threads, device_m05=dev)
    t = time.perf_counter()
    outs, st = vp8g.gpu_decode_webp_batch(batch, True, threads, device_m05=dev)
    dt = vp8g.gpu_decode_webp_batch.seconds  # the C call: .webp bytes -> I420 images
    ok = all(s == 0 for s in st) and all(
        hashlib.sha256(outs[i]).hexdigest() == man["files"][FIXTURES[i % 4]]["yuvf_sha256"] for i in range(n))
    print(json.dumps({"device_m05": dev, "frames": n, "threads": threads, "seconds": round(dt, 3),
                      "MP/s": round(n * 3840 * 2160 / 1e6 / dt, 1), "ok": ok}), flush=True)
