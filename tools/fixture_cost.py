#!/usr/bin/env python3
"""Per-fixture decode cost in chain mode (diagnostics for the chain planner's cost model).

Each 4K / 1080p fixture is replicated into a batch of its own (512 x 4K, 2048 x 1080p: every CU
holds frames of one kind) and `vp8g_decode_batch_device` is timed; cost = kernel ms x CUs / frames
(CU-ms per frame).  Printed beside the host-side content features the model can use (MBs, B_PRED
MBs, blocks with AC, non-zero coefficients, MBs with coefficients, loop-filter parameters).

  python tools/fixture_cost.py [--libs lib.so]   ->   one JSON line per fixture
"""
import argparse
import ctypes as C
import json
import pathlib
import statistics
import sys

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "webp-decoder_amd"))

UHD = ["big/uhd_a_normal_seg4.webp", "big/uhd_b_simple_sharp3.webp", "big/uhd_c_normal_sharp6_seg1.webp",
       "big/uhd_d_normal_q90.webp"]
FHD = ["big/fhd_normal_sharp5.webp", "big/fhd_simple_sharp3.webp", "big/fhd_c_normal_q85_seg4.webp",
       "big/fhd_d_normal_sharp2_seg1.webp"]


def features(f, d):
    import vp8g  # noqa: F401
    n = f.mb_total
    y = f.array("coeff_y").reshape(n, 16, 16)
    u = f.array("coeff_u").reshape(n, 4, 16)
    v = f.array("coeff_v").reshape(n, 4, 16)
    blk = np.concatenate([y, u, v], axis=1)
    lf = np.ctypeslib.as_array(d.lf).reshape(4, 2, 4)
    return {"mbs": n, "bpred": int((f.array("ymode") == 4).sum()), "ac_blocks": int((blk[:, :, 1:] != 0).any(axis=2).sum()),
            "nnz": int((blk != 0).sum() + (f.array("coeff_y2") != 0).sum()), "has_coeff": int((f.array("has_coeff") != 0).sum()),
            "lf": lf[:, :, :3].tolist(), "flags": int(d.flags)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=6)
    a = ap.parse_args()
    import torch
    import vp8g
    import vp8g_batch
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    cus = torch.cuda.get_device_properties(dev).multi_processor_count
    stream = torch.cuda.current_stream(dev).cuda_stream
    for rel, n in [(r, 512) for r in UHD] + [(r, 2048) for r in FHD]:
        f = vp8g.decode_file(ROOT / "tests" / "fixtures" / rel)
        b = vp8g_batch.DeviceBatch(n, f.width, f.height, dev)
        b.replicate([f], True)
        b.commit()
        b.launch(stream)
        torch.cuda.synchronize()
        ts = []
        for _ in range(a.steps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            b.launch(stream)
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1))
        ms = statistics.median(ts)
        print(json.dumps({"fixture": rel, "frames": n, "kernel_ms": round(ms, 3), "cu_ms_per_frame": round(ms * cus / n, 3),
                          **features(f, b.h_descs[0])}), flush=True)
        del b
        f.free()
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
