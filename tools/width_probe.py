#!/usr/bin/env python3
"""Kernel time of synthetic 4K-class batches by frame width (diagnostics): 3840 (whole pieces: the
quad kernel's paired instantiation) against widths that cut the last MB column and leave every
other luma row 8-B aligned (3832, 3848: the general instantiation), 64 distinct frames replicated
to n slots; a few slots are checked against the oracle.
  python tools/width_probe.py [n] [widths...]"""
import pathlib
import sys
import time

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "webp-decoder_amd"))
import torch  # noqa: E402
import vp8g  # noqa: E402
import vp8g_batch  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 512
widths = [int(w) for w in sys.argv[2:]] or [3840, 3832, 3848]
dev = torch.device("cuda:0")
stream = torch.cuda.current_stream(dev).cuda_stream
for W in widths:
    frames = [vp8g.synth_frame(W, 2160, 0x7A11 ^ (i * 977), profile=i % 3) for i in range(16)]
    b = vp8g_batch.DeviceBatch(n, W, 2160, dev)
    b.replicate(frames, True)
    b.commit()
    ts = []
    for _ in range(7):
        torch.cuda.synchronize()
        t = time.perf_counter()
        b.launch(stream)
        torch.cuda.synchronize()
        ts.append((time.perf_counter() - t) * 1e3)
    bad = [i for i in (0, 5, n - 1) if b.frame_output(i) != vp8g.oracle_reconstruct(frames[i % 16], True)]
    ts.sort()
    print(f"W={W} mode={b.launch_mode()} median_ms={ts[3]:.3f} min_ms={ts[0]:.3f} status={b.status_word()} "
          f"oracle_mismatch={bad}", flush=True)
    for f in frames:
        f.free()
    del b
    torch.cuda.empty_cache()
