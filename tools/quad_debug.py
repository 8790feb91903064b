#!/usr/bin/env python3
"""Where two libvp8g builds disagree (diagnostics for experiment kernels): one launch of each on the
same batch, then per frame the MBs whose Y / U / V pixels differ.

  python tools/quad_debug.py [--workload uhd4_yuv] [--frames 512] ref.so test.so
"""
import argparse
import ctypes as C
import json
import pathlib
import sys

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "webp-decoder_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="uhd4_yuv")
    ap.add_argument("--frames", type=int, default=0)
    ap.add_argument("--show", type=int, default=3, help="frames to detail")
    ap.add_argument("libs", nargs=2)
    a = ap.parse_args()
    import torch
    import bench
    import vp8g
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    golden = json.loads((ROOT / "tests" / "golden" / "digests.json").read_text())
    args = bench.parse(["--workload", a.workload, "--frames", str(a.frames), "--no-cpu-baseline"])
    r = bench.Rank(a.workload, args, 0, 1, dev, golden, None)
    b = r.batch
    stream = torch.cuda.current_stream(dev).cuda_stream
    outs, stats = [], []
    for path in a.libs:
        lib = C.CDLL(str(pathlib.Path(path).resolve()), use_errno=True)
        lib.vp8g_decode_batch_device.argtypes = [C.POINTER(vp8g.Vp8gFrameDesc), C.c_void_p, C.c_uint32,
                                                 C.POINTER(vp8g.Vp8gBatchArrays), C.c_void_p, C.c_void_p, C.c_uint32]
        lib.vp8g_last_error.restype = C.c_char_p
        b.out.fill_(0xA5)
        b.status.zero_()
        rc = lib.vp8g_decode_batch_device(b.h_descs, C.c_void_p(b.d_descs.data_ptr()), b.n, C.byref(b.c_arrays),
                                          C.c_void_p(b.out.data_ptr()), C.c_void_p(stream), 0)
        torch.cuda.synchronize()
        if rc != 0:
            raise RuntimeError(lib.vp8g_last_error())
        outs.append(b.out.cpu().numpy().copy())
        stats.append(int(b.status[0].item()))
    print("status", stats, flush=True)
    ref, tst = outs
    bad_frames = []
    for i in range(b.n):
        d = b.h_descs[i]
        o = i * b.frame_bytes
        if not np.array_equal(ref[o:o + b.i420], tst[o:o + b.i420]):
            bad_frames.append(i)
    print(f"frames differing: {len(bad_frames)} of {b.n}; first {bad_frames[:16]}", flush=True)
    for i in bad_frames[:a.show]:
        d = b.h_descs[i]
        o = i * b.frame_bytes
        W, H, sy, suv = d.width, d.height, d.stride_y, d.stride_uv
        cw, ch = (W + 1) // 2, (H + 1) // 2
        R, Cc = d.mb_rows, d.mb_cols
        bad = np.zeros((R, Cc, 3), bool)
        first = None
        for p, (off, stride, pw, ph, s) in enumerate([(d.out_y, sy, W, H, 16), (d.out_u, suv, cw, ch, 8), (d.out_v, suv, cw, ch, 8)]):
            A = ref[o + off:o + off + stride * ph].reshape(ph, stride)[:, :pw]
            B = tst[o + off:o + off + stride * ph].reshape(ph, stride)[:, :pw]
            diff = A != B
            ys, xs = np.nonzero(diff)
            for y, x in zip(ys, xs):
                bad[y // s, x // s, p] = True
            if len(ys) and first is None:
                first = (p, int(ys[0]), int(xs[0]), int(A[ys[0], xs[0]]), int(B[ys[0], xs[0]]))
        anyb = bad.any(axis=2)
        rows = [(rr, int(anyb[rr].sum()), [int(x) for x in np.nonzero(anyb[rr])[0][:8]]) for rr in range(R) if anyb[rr].any()]
        print(f"frame {i}: {int(anyb.sum())} of {R * Cc} MBs differ; first pixel (plane, y, x, ref, test) {first}")
        print("  rows (row, count, first cols):", rows[:24])
        print("  row mod 4 counts:", [int(anyb[rr::4].sum()) for rr in range(4)], " planes:", [int(bad[:, :, p].sum()) for p in range(3)])


if __name__ == "__main__":
    main()
