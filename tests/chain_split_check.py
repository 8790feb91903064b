"""Helper of tests/test_gpu_batch.py::test_chain_mirror_split_forced (run in a child process with
VP8G_SPLITCHAIN=1, read once by libvp8g): the chain test's mixed small-frame batch (~7 frames per
workgroup, so every workgroup's list holds many top and bottom segments) decoded with every frame
of more than two MB rows split between two workgroups, each slot against the oracle."""
import pathlib
import sys

import numpy as np
import torch

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "webp-decoder_amd"))
import vp8g  # noqa: E402
import vp8g_batch  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    rng = np.random.default_rng(23)
    sizes = [(1, 1), (16, 48), (17, 9), (160, 64), (33, 47), (160, 96), (1024, 80), (8, 96), (1000, 40)]
    frames = [vp8g.synth_frame(*sizes[i % len(sizes)], 0x5B17 ^ i, profile=i % 3) for i in range(36)]
    n = 1500
    b = vp8g_batch.DeviceBatch(n, 1024, 96, dev)
    b.out.fill_(0xA5)
    pick = rng.integers(0, len(frames), n)
    for i in range(n):
        b.place(i, frames[pick[i]], bool(pick[i] % 2))
    b.commit()
    stream = torch.cuda.current_stream(dev).cuda_stream
    for rep in range(2):  # (a second launch reuses the snapshot flags with the next epoch)
        b.launch(stream)
        torch.cuda.synchronize()
        assert b.status_word() == 0, b.status_word()
    exp, bad = {}, []
    for i in range(n):
        j = int(pick[i])
        key = (j, bool(j % 2))
        if key not in exp:
            exp[key] = vp8g.oracle_reconstruct(frames[j], bool(j % 2))
        if b.frame_output(i)[:len(exp[key])] != exp[key]:
            bad.append(i)
    print("OK" if not bad else f"BAD {len(bad)} of {n}: {bad[:8]}")


if __name__ == "__main__":
    main()
