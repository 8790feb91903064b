"""Device m05 kernel time vs batch size (one 3840x2160 fixture repeated), HIP events around the
launch.  Usage: python tools/m05_kernel_probe.py [fixture-index 0..3] [N ...]"""
import ctypes as C
import json
import os
import pathlib
import sys

import numpy as np
import torch

ROOT = pathlib.Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "webp-decoder_amd"))
sys.path.insert(0, str(ROOT))
import vp8g  # noqa: E402
from bench import FIXTURES  # noqa: E402

fi = int(sys.argv[1]) if len(sys.argv) > 1 else 0
ns = [int(a) for a in sys.argv[2:]] or [1, 64, 256, 1024]
data = (ROOT / "tests" / "fixtures" / FIXTURES[fi]).read_bytes()
log2k = int(os.environ.get("M05_LOG2K", "0"))  # re-encode over 2^k token partitions (test generator)
if log2k:
    sys.path.insert(0, str(ROOT / "tests"))
    from multipart import repartition  # noqa: E402
    data = repartition(data, log2k)
kf, hdr, tf, off, size = vp8g.token_header(data, multi_partition=log2k > 0)
lib = vp8g.gpu_lib()
dev = torch.device("cuda:0")
slot = (size + 512 + 15) & ~15
mb = hdr.mb_total
for n in ns:
    bits = np.zeros(slot * n, np.uint8)
    jobs = (vp8g.Vp8gTokFrame * n)()
    for i in range(n):
        bits[i * slot:i * slot + size] = np.frombuffer(data, np.uint8, size, off)
        jobs[i] = tf
        jobs[i].data, jobs[i].mb_offset = i * slot, i * mb
    d_bits = torch.from_numpy(bits).to(dev)
    d_jobs = torch.from_numpy(np.frombuffer(bytes(jobs), np.uint8).copy()).to(dev)
    arr_t = {k: torch.zeros(n * mb * per, dtype=torch.int16 if dt == np.int16 else torch.uint8, device=dev)
             for k, dt, per in vp8g.FRAME_ARRAYS if k != "skip_coeff"}
    st = torch.zeros(1, dtype=torch.int32, device=dev)
    arr = vp8g.Vp8gBatchArrays(**{k: v.data_ptr() for k, v in arr_t.items()}, src=None, status=st.data_ptr())
    times = []
    for rep in range(2):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record()
        assert lib.vp8g_m05_batch_device(jobs, d_jobs.data_ptr(), n, d_bits.data_ptr(), C.byref(arr), None) == 0
        e1.record()
        torch.cuda.synchronize()
        times.append(e0.elapsed_time(e1))
    ms = min(times)
    print(json.dumps({"fixture": FIXTURES[fi], "partitions": 1 << log2k, "payload_bytes": size, "frames": n, "ms": round(ms, 2),
                      "frames_per_s": round(n / ms * 1e3, 1), "MB_per_s_compressed": round(n * size / ms / 1e3, 1),
                      "MP_per_s": round(n * 3840 * 2160 / ms / 1e3, 1)}), flush=True)
    del d_bits, d_jobs, arr_t
