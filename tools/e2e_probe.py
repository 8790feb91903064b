#!/usr/bin/env python3
"""End-to-end device-m05 timing probe (diagnostics): the bench's 1024-frame leg in a fresh process,
then with device memory held by torch (as inside bench.py), with VP8G_PIPE_TRACE=1 chunk traces."""
import os, pathlib, sys
import torch  # before libvp8g: torch must initialise the device first in this process
ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "webp-decoder_amd"))
import vp8g
UHD = ["big/uhd_a_normal_seg4.webp", "big/uhd_b_simple_sharp3.webp", "big/uhd_c_normal_sharp6_seg1.webp", "big/uhd_d_normal_q90.webp"]
files = [(ROOT / "tests" / "fixtures" / r).read_bytes() for r in UHD]
thr = int(os.environ.get("OMP_NUM_THREADS", "16"))
n = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
hold = int(sys.argv[2]) if len(sys.argv) > 2 else 40
os.environ["VP8G_PIPE_TRACE"] = "1"
torch.zeros(1, device="cuda")
vp8g.gpu_decode_webp_batch(files * 2, True, thr, device_m05=True)
batch = [files[i % 4] for i in range(n)]
def run(tag):
    outs, st = vp8g.gpu_decode_webp_batch(batch, True, thr, device_m05=True)
    assert all(s == 0 for s in st)
    print(f"== {tag}: {vp8g.gpu_decode_webp_batch.seconds:.3f} s", file=sys.stderr, flush=True)
run("fresh")
run("fresh again")
x = torch.empty(hold << 30, dtype=torch.uint8, device="cuda")
run(f"with {hold} GiB held")
del x
torch.cuda.empty_cache()
os.environ["VP8G_HYBRID"] = "0"
run("hybrid off")
