#!/usr/bin/env python3
"""Co-resident frame pairing probe (diagnostics): the same device batch launched with its frame
descriptors in different orders.  Workgroups b and b + 256 share a CU (profiles/r02b_wave_placement.json),
so the order decides which two frames run side by side.  uhd4 replicates 4 fixtures round-robin,
which pairs every frame with a copy of itself; the permutations below pair them differently.
Prints per order the median kernel ms (interleaved rounds) and digest parity.

  python tools/pair_probe.py [--workload uhd4] [--rounds 6] [--steps 8]
"""
import argparse
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
    ap.add_argument("--rounds", type=int, default=6)
    ap.add_argument("--steps", type=int, default=8)
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
    n = b.n
    half = n // 2
    lib = vp8g.gpu_lib()
    stream = torch.cuda.current_stream(dev).cuda_stream
    fix = r.param_index  # fixture index of each slot

    def partner_perm(mapf):
        """slots >= half get the slot of the same group of 4 whose fixture is mapf(own fixture)"""
        perm = list(range(n))
        for j in range(half, n):
            base = j - (j % 4)
            want = mapf(fix[j])
            perm[j] = next(base + q for q in range(4) if fix[base + q] == want)
        assert sorted(perm) == list(range(n))
        return perm

    orders = {"identity": list(range(n)),
              "a-d,b-c": partner_perm(lambda f: 3 - f),
              "a-b,c-d": partner_perm(lambda f: f ^ 1),
              "a-c,b-d": partner_perm(lambda f: f ^ 2)}
    inst = {}
    for name, perm in orders.items():
        h = (vp8g.Vp8gFrameDesc * n)()
        for j, i in enumerate(perm):
            h[j] = b.h_descs[i]
        d = torch.frombuffer(bytearray(bytes(h)), dtype=torch.uint8).to(dev)
        inst[name] = (perm, h, d)

    def launch(h, d):
        rc = lib.vp8g_decode_batch_device(h, C.c_void_p(d.data_ptr()), n, C.byref(b.c_arrays),
                                          C.c_void_p(b.out.data_ptr()), C.c_void_p(stream), 0)
        if rc != 0:
            raise RuntimeError(f"launch failed: {lib.vp8g_last_error()!r}")

    times = {k: [] for k in orders}
    parity = {}
    for rnd in range(a.rounds):
        for name, (perm, h, d) in inst.items():
            launch(h, d)
            torch.cuda.synchronize()
            evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(a.steps)]
            for s in range(a.steps):
                evs[s][0].record()
                launch(h, d)
                evs[s][1].record()
            torch.cuda.synchronize()
            times[name] += [x.elapsed_time(y) for x, y in evs]
            if rnd == 0:
                b.status.zero_()
                b.out.zero_()
                launch(h, d)
                dig = b.digests(stream)  # in the batch's own slot order
                exp = [r.expected_for(r.lo + i) for i in range(n)]
                parity[name] = sum(int(x) == int(e, 16) for x, e in zip(dig, exp) if e)
    for name in orders:
        t = times[name]
        print(json.dumps({"order": name, "median_ms": round(statistics.median(t), 3), "min_ms": round(min(t), 3),
                          "parity": f"{parity[name]}/{n}"}), flush=True)


if __name__ == "__main__":
    main()
