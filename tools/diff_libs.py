#!/usr/bin/env python3
"""Byte-level difference of two libvp8g builds on one device batch (diagnostics).

Runs the bench workload batch through `vp8g_decode_batch_device` of each library and reports, for
the first differing slot, which planes / rows / columns differ (row and column residues mod 16 and
the MB coordinates), so a kernel change that breaks parity can be located without a debugger.

  python tools/diff_libs.py [--workload uhd4] [--frames 8] good.so bad.so
"""
import argparse
import collections
import ctypes as C
import pathlib
import sys

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "webp-decoder_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="uhd4")
    ap.add_argument("--frames", type=int, default=8)
    ap.add_argument("libs", nargs=2)
    a = ap.parse_args()
    import torch
    import bench
    import vp8g
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    args = bench.parse(["--workload", a.workload, "--frames", str(a.frames), "--no-cpu-baseline"])
    import json
    golden = json.loads((ROOT / "tests" / "golden" / "digests.json").read_text())
    r = bench.Rank(a.workload, args, 0, 1, dev, golden, None)
    b = r.batch
    stream = torch.cuda.current_stream(dev).cuda_stream
    outs = []
    for path in a.libs:
        lib = C.CDLL(str(pathlib.Path(path).resolve()), use_errno=True)
        lib.vp8g_decode_batch_device.argtypes = [C.POINTER(vp8g.Vp8gFrameDesc), C.c_void_p, C.c_uint32,
                                                 C.POINTER(vp8g.Vp8gBatchArrays), C.c_void_p, C.c_void_p, C.c_uint32]
        b.out.fill_(0xA5)
        b.status.zero_()
        rc = lib.vp8g_decode_batch_device(b.h_descs, C.c_void_p(b.d_descs.data_ptr()), b.n, C.byref(b.c_arrays),
                                          C.c_void_p(b.out.data_ptr()), C.c_void_p(stream), 0)
        torch.cuda.synchronize()
        print(path, "rc", rc, "status", int(b.status.item()) if b.status.numel() == 1 else b.status.cpu().tolist())
        outs.append(b.out.cpu().numpy().copy())
    x, y = outs
    for i in range(b.n):
        d = b.h_descs[i]
        W, H = int(d.width), int(d.height)
        CW, CH = (W + 1) // 2, (H + 1) // 2
        planes = [("Y", int(d.out_y), int(d.stride_y), W, H), ("U", int(d.out_u), int(d.stride_uv), CW, CH),
                  ("V", int(d.out_v), int(d.stride_uv), CW, CH)]
        bad = False
        for name, off, st, w, h in planes:
            px = x[off:off + st * h].reshape(h, st)[:, :w]
            py = y[off:off + st * h].reshape(h, st)[:, :w]
            diff = np.argwhere(px != py)
            if len(diff) == 0:
                continue
            bad = True
            mb = 16 if name == "Y" else 8
            rows = collections.Counter((diff[:, 0] % mb).tolist())
            cols = collections.Counter((diff[:, 1] % mb).tolist())
            mbr = collections.Counter((diff[:, 0] // mb).tolist())
            mbc = collections.Counter((diff[:, 1] // mb).tolist())
            print(f"slot {i} plane {name}: {len(diff)} of {w * h} bytes differ")
            print("  row%mb:", sorted(rows.items())[:20])
            print("  col%mb:", sorted(cols.items())[:20])
            print("  MB rows (first 12):", sorted(mbr.items())[:12], "... MB cols (first 12):", sorted(mbc.items())[:12])
            print("  first diffs (row, col, good, bad):", [(int(r_), int(c_), int(px[r_, c_]), int(py[r_, c_])) for r_, c_ in diff[:12]])
        if bad:
            break
    else:
        print("identical")


if __name__ == "__main__":
    main()
