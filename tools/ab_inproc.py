#!/usr/bin/env python3
"""Interleaved in-process A/B timing of several libvp8g builds on ONE device batch (diagnostics).

The batch (bench workload, default uhd4) is built once; every library is loaded side by side
(ctypes, RTLD_LOCAL: each handle resolves its own kernels) and timed in rounds, so box-to-box and
setup variation drop out.  Each entry is `path[:waves]`.  Prints per library the median kernel ms
over all rounds and whether its digests match the golden ones.

  python tools/ab_inproc.py [--workload uhd4] [--rounds 5] [--steps 8] lib1.so lib2.so:10 ...
"""
import argparse
import hashlib
import ctypes as C
import json
import pathlib
import statistics
import sys

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "webp-decoder_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="uhd4")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--steps", type=int, default=8)
    ap.add_argument("--frames", type=int, default=0)
    ap.add_argument("libs", nargs="+")
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
    libs = []
    for ent in a.libs:
        path, _, w = ent.partition(":")
        lib = C.CDLL(str(pathlib.Path(path).resolve()), use_errno=True)
        lib.vp8g_decode_batch_device.argtypes = [C.POINTER(vp8g.Vp8gFrameDesc), C.c_void_p, C.c_uint32,
                                                 C.POINTER(vp8g.Vp8gBatchArrays), C.c_void_p, C.c_void_p, C.c_uint32]
        lib.vp8g_last_error.restype = C.c_char_p
        lib.vp8g_frame_digests.argtypes = [C.POINTER(vp8g.Vp8gFrameDesc), C.c_void_p, C.c_uint32, C.c_void_p,
                                           C.c_void_p, C.c_void_p]
        libs.append((ent, lib, int(w or 0)))

    def launch(lib, waves):
        rc = lib.vp8g_decode_batch_device(b.h_descs, C.c_void_p(b.d_descs.data_ptr()), b.n, C.byref(b.c_arrays),
                                          C.c_void_p(b.out.data_ptr()), C.c_void_p(stream), waves)
        if rc != 0:
            raise RuntimeError(f"launch failed: {lib.vp8g_last_error()!r}")

    times = {e: [] for e, _, _ in libs}
    parity, outhash = {}, {}
    for rnd in range(a.rounds):
        for ent, lib, w in libs:
            launch(lib, w)
            torch.cuda.synchronize()
            evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(a.steps)]
            for s in range(a.steps):
                evs[s][0].record()
                launch(lib, w)
                evs[s][1].record()
            torch.cuda.synchronize()
            times[ent] += [x.elapsed_time(y) for x, y in evs]
            if rnd == 0:
                b.status.zero_()
                launch(lib, w)
                dig = b.digests(stream)
                exp = [r.expected_for(r.lo + i) for i in range(b.n)]
                parity[ent] = sum(int(d) == int(e, 16) for d, e in zip(dig, exp) if e)
                # (unpinned workloads: builds are compared with each other through this hash)
                outhash[ent] = hashlib.sha256(dig.tobytes()).hexdigest()[:16]
    for ent, _, _ in libs:
        t = times[ent]
        print(json.dumps({"lib": ent, "median_ms": round(statistics.median(t), 3), "min_ms": round(min(t), 3),
                          "parity": f"{parity[ent]}/{b.n}", "digests_sha": outhash[ent]}), flush=True)


if __name__ == "__main__":
    main()
