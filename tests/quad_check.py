"""Batch decoded by the quad chain kernel (csrc/vp8g_quad.inc: four MB rows per wave; every chain
batch without loop-filter-only frames), every slot against the oracle.  Imported by tests/test_gpu_quad.py,
and run as a child process there when an environment switch read once by libvp8g must be set
(VP8G_SPLITCHAIN=1: every frame of more than four MB rows split between two workgroups).

Frames (SIZES): widths multiples of 16 (whole 16-B / 8-B row pieces: the kernel's lean instantiation),
heights giving 1..19 MB rows -- last quads of one, two, three and four rows -- and odd pixel heights
(cropped bottom rows); ODD_SIZES adds widths that cut the right MB's pieces and rows that start
unaligned (stride = width: the general instantiation's byte path).  All synthetic
profiles (segments, loop-filter deltas, simple and normal filter, +-2114 coefficients), filtered and
unfiltered, in a scrambled order with one slot in eight left empty."""
import pathlib
import sys

import numpy as np
import torch

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "webp-decoder_amd"))
import vp8g  # noqa: E402
import vp8g_batch  # noqa: E402

SIZES = [(16, 16), (16, 48), (32, 24), (160, 64), (48, 112), (1024, 80), (160, 96), (64, 200), (128, 304), (96, 36)]
ODD_SIZES = SIZES[:5] + [(1, 1), (17, 16), (33, 50), (100, 70), (250, 130), (1000, 37), (8, 8), (24, 200), (52, 300), (15, 33)]


def run(n=1800, seed=0x0A4D, launches=1, want_split=False, sizes=SIZES):
    dev = torch.device("cuda:0")
    rng = np.random.default_rng(seed)
    frames = [vp8g.synth_frame(*sizes[i % len(sizes)], seed ^ (i * 0x9E37), profile=i % 3) for i in range(40)]
    W = max(w for w, _ in sizes)
    H = max(h for _, h in sizes)
    b = vp8g_batch.DeviceBatch(n, W, H, dev)
    b.out.fill_(0xA5)
    pick = rng.integers(0, len(frames), n)
    empty = set(rng.choice(n, n // 8, replace=False).tolist())
    for i in range(n):
        if i not in empty:
            b.place(i, frames[pick[i]], bool(pick[i] % 2))
    b.commit()
    stream = torch.cuda.current_stream(dev).cuda_stream
    for _ in range(launches):
        b.launch(stream)
        torch.cuda.synchronize()
        if b.status_word() != 0:
            return [f"status {b.status_word()}"]
        mode = b.launch_mode()
        if not (mode & vp8g.MODE_CHAIN and mode & vp8g.MODE_QUAD) or (want_split and not mode & vp8g.MODE_MIRROR_SPLIT):
            return [f"launch mode {mode}: not the quad chain{' with the mirror split' if want_split else ''}"]
    exp, bad = {}, []
    for i in range(n):
        if i in empty:
            continue
        j = int(pick[i])
        key = (j, bool(j % 2))
        if key not in exp:
            exp[key] = vp8g.oracle_reconstruct(frames[j], bool(j % 2))
        if b.frame_output(i)[:len(exp[key])] != exp[key]:
            bad.append(i)
    for i in sorted(empty)[:16]:
        if b.frame_output(i) != b"\xa5" * b.i420:
            bad.append(f"empty slot {i} written")
    for f in frames:
        f.free()
    return bad


if __name__ == "__main__":
    import os
    bad = run(launches=2, want_split=os.environ.get("VP8G_SPLITCHAIN") == "1",
              sizes=ODD_SIZES if "--odd" in sys.argv else SIZES)
    print("OK" if not bad else f"BAD {len(bad)}: {bad[:8]}")
