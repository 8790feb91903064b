#!/usr/bin/env python3
"""Where frame_kernel's waves run and when they end (diagnostics; stamps builds only).

Loads a VP8G_STAMPS build, launches the bench batch once, reads per-wave {HW_ID, XCC_ID,
duration} of blocks < 512 (vp8g_debug_wave_info) and prints: mean wave duration by wave index,
how many of each CU's 'long' waves (those handling the most row pairs) share a SIMD, and the
spread of block durations.
  python tools/wave_tail.py lib.so [--workload uhd4]
"""
import argparse, collections, ctypes as C, json, pathlib, statistics, sys
ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT)); sys.path.insert(0, str(ROOT / "webp-decoder_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("lib")
    ap.add_argument("--workload", default="uhd4")
    a = ap.parse_args()
    import torch
    import bench
    import vp8g
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    golden = json.loads((ROOT / "tests" / "golden" / "digests.json").read_text())
    args = bench.parse(["--workload", a.workload, "--no-cpu-baseline"])
    r = bench.Rank(a.workload, args, 0, 1, dev, golden, None)
    b = r.batch
    lib = C.CDLL(str(pathlib.Path(a.lib).resolve()))
    lib.vp8g_decode_batch_device.argtypes = [C.POINTER(vp8g.Vp8gFrameDesc), C.c_void_p, C.c_uint32,
                                             C.POINTER(vp8g.Vp8gBatchArrays), C.c_void_p, C.c_void_p, C.c_uint32]
    stream = torch.cuda.current_stream(dev).cuda_stream
    for _ in range(3):
        assert lib.vp8g_decode_batch_device(b.h_descs, C.c_void_p(b.d_descs.data_ptr()), b.n, C.byref(b.c_arrays),
                                            C.c_void_p(b.out.data_ptr()), C.c_void_p(stream), 0) == 0
    torch.cuda.synchronize()
    buf = (C.c_ulonglong * (512 * 16 * 2))()
    assert lib.vp8g_debug_wave_info(buf) == 0
    nb = min(512, b.n)
    dur = collections.defaultdict(list)
    cu_waves = collections.defaultdict(list)
    blk = []
    for bi in range(nb):
        ws = []
        for w in range(16):
            if buf[2 * (bi * 16 + w) + 1] == 0:  # (8-wave workgroups record waves 0..7 only)
                continue
            hw = buf[2 * (bi * 16 + w)]
            d = buf[2 * (bi * 16 + w) + 1] / 100.0  # us (100 MHz)
            simd, cu, sh, se, xcc = (hw >> 4) & 3, (hw >> 8) & 15, (hw >> 12) & 1, (hw >> 13) & 7, (hw >> 32) & 15
            dur[w].append(d)
            ws.append(d)
            cu_waves[(xcc, se, sh, cu)].append((bi, w, simd, d))
        if ws:  # (chain mode: one block per CU, fewer blocks than frames)
            blk.append(max(ws))
    print("mean duration by wave (us):", {w: round(statistics.mean(v), 1) for w, v in sorted(dur.items())})
    print("block duration (us): median %.1f max %.1f min %.1f" % (statistics.median(blk), max(blk), min(blk)))
    q = sorted(blk)
    print("block duration deciles (us):", [round(q[min(len(q) - 1, int(len(q) * k / 10))], 1) for k in range(11)])
    if r.wl["kind"] == "fixtures" and len(blk) == nb:  # slot i holds fixture i mod len(fixtures)
        nf = len(r.wl["fixtures"])
        print("block duration by fixture (us, median):",
              {r.wl["fixtures"][k]: round(statistics.median(blk[k::nf]), 1) for k in range(nf)})
    long_share = collections.Counter()
    simd_last = []
    for key, v in cu_waves.items():
        v.sort(key=lambda t: -t[3])
        top = v[:4]  # the four longest waves on this CU
        long_share[tuple(sorted(collections.Counter(t[2] for t in top).values()))] += 1
        per_simd = collections.defaultdict(float)
        for t in v:
            per_simd[t[2]] = max(per_simd[t[2]], t[3])
        simd_last.append(sorted(per_simd.values()))
    print("the 4 longest waves of a CU per SIMD (multiset of counts -> CUs):", dict(long_share))
    print("per CU, last wave end per SIMD (us, mean over CUs, sorted):",
          [round(statistics.mean(x[i] for x in simd_last), 1) for i in range(4)])


if __name__ == "__main__":
    main()
