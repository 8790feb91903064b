"""GPU: the quad chain kernel (csrc/vp8g_quad.inc) -- four MB rows per wave, the
row above a quad handed over through device memory, progress published one step late -- on the
shapes the bench batches do not have.  Reference path: src/m06_recon/vp8_recon.c:444-684 (MB
driver) + src/m07_loopfilter/vp8_loopfilter.c:214-280 (filter order), per frame."""
import os
import subprocess
import sys

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu


def test_quad_chain_mixed_whole_piece_frames(vp8g):
    """1 800 slots (~7 frames per workgroup) of 40 distinct whole-piece frames, 1..19 MB rows (last
    quads of 1, 2, 3 and 4 rows), cropped heights, filtered and unfiltered, one slot in eight empty:
    every decoded slot equals the oracle's output, the empty slots stay untouched."""
    sys.path.insert(0, str(ROOT / "tests"))
    import quad_check
    bad = quad_check.run()
    assert not bad, f"{len(bad)} slots differ, e.g. {bad[:8]}"


def test_quad_chain_cut_and_unaligned_pieces(vp8g):
    """Widths that are not multiples of 16 (1, 8, 15, 17, 33, 52, 100, 250, 1000) mixed with
    whole-piece frames: the right MB's row pieces are cut and rows start unaligned (stride = width),
    so the batch takes the quad kernel's general instantiation (byte path for those pieces); every
    slot equals the oracle's output, the empty slots stay untouched."""
    sys.path.insert(0, str(ROOT / "tests"))
    import quad_check
    bad = quad_check.run(n=1200, seed=0x0DD5, sizes=quad_check.ODD_SIZES)
    assert not bad, f"{len(bad)} slots differ, e.g. {bad[:8]}"


@pytest.mark.parametrize("odd", [False, True])
def test_quad_chain_mirror_split_forced(vp8g, odd):
    """The same kinds of batch with the mirror split forced (VP8G_SPLITCHAIN=1, child process): a
    bottom segment's first quad reads the frame's context from device memory after the top
    segment's flag; two launches (the flags' epoch advances)."""
    env = dict(os.environ, VP8G_SPLITCHAIN="1")
    r = subprocess.run([sys.executable, str(ROOT / "tests" / "quad_check.py")] + (["--odd"] if odd else []), capture_output=True,
                       text=True, timeout=240, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    assert r.stdout.strip().endswith("OK"), r.stdout


def test_quad_and_pairs_chains_agree(vp8g):
    """260 x 4K fixtures (slot i <- fixture i % 4) through the quad chain and, in a child process with
    VP8G_QUAD=0, through the two-rows-per-wave chain: both equal the reference's digests."""
    code = r"""
import json, pathlib, sys
root = pathlib.Path(sys.argv[1])
sys.path.insert(0, str(root / "webp-decoder_amd"))
import torch, vp8g, vp8g_batch
UHD = ["big/uhd_a_normal_seg4.webp", "big/uhd_b_simple_sharp3.webp", "big/uhd_c_normal_sharp6_seg1.webp",
       "big/uhd_d_normal_q90.webp"]
golden = json.loads((root / "tests" / "golden" / "digests.json").read_text())
dev = torch.device("cuda:0")
frames = [vp8g.decode_file(root / "tests" / "fixtures" / r) for r in UHD]
b = vp8g_batch.DeviceBatch(260, 3840, 2160, dev)
b.replicate(frames, True)
b.commit()
stream = torch.cuda.current_stream(dev).cuda_stream
b.launch(stream)
dig = b.digests(stream)
bad = [i for i in range(260) if int(dig[i]) != int(golden["fixtures"][UHD[i % 4]]["yuvf"], 16)]
mode = b.launch_mode()
print(mode, "OK" if not bad and b.status_word() == 0 else f"BAD {bad[:8]} status {b.status_word()}")
"""
    for env_extra in ({}, {"VP8G_QUAD": "0"}):
        env = dict(os.environ, **env_extra)
        r = subprocess.run([sys.executable, "-c", code, str(ROOT)], capture_output=True, text=True, timeout=240, env=env)
        assert r.returncode == 0, (env_extra, r.stderr[-2000:])
        assert r.stdout.strip().endswith("OK"), (env_extra, r.stdout)
        mode = int(r.stdout.split()[0])
        quad = env_extra.get("VP8G_QUAD") != "0"
        assert mode & vp8g.MODE_CHAIN and bool(mode & vp8g.MODE_QUAD) == quad, (env_extra, mode)


def test_quad_chain_stalled_producer_ends_promptly(vp8g):
    """A quad chain whose wave 1 never publishes its progress (libvp8g_stall.so: wait bound 20 ms):
    the waits are bounded and sticky, so the launch ends promptly with the timeout bit in the status
    word instead of hanging the chain (the quad's progress is published one step late, and its first
    step's context load waits too -- every wait path bounded).  Frames of 128 MB rows: 16 quads per
    mirror-split segment, so wave 1's units have successors that wait on its progress whatever the
    schedule."""
    code = r"""
import ctypes as C, sys, time
sys.path.insert(0, sys.argv[1] + "/webp-decoder_amd")
import torch, vp8g, vp8g_batch
vp8g._libs["gpu"] = C.CDLL(sys.argv[1] + "/webp-decoder_amd/lib/diag/libvp8g_stall.so", use_errno=True)
dev = torch.device("cuda:0")
cus = torch.cuda.get_device_properties(0).multi_processor_count
n = 2 * cus
frames = [vp8g.synth_frame(160, 2048, 0x5A11 ^ i, profile=i % 3) for i in range(8)]
b = vp8g_batch.DeviceBatch(n, 160, 2048, dev)
for i in range(n):
    b.fill(i, frames[i % 8], True)
b.commit()
stream = torch.cuda.current_stream(dev).cuda_stream
t = time.time()
b.launch(stream)
torch.cuda.synchronize()
print(b.status_word(), b.launch_mode(), round(time.time() - t, 3))
"""
    r = subprocess.run([sys.executable, "-c", code, str(ROOT)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    status, mode, secs = r.stdout.split()[-3:]
    assert int(status) & 1, r.stdout  # VP8G_ERR_TIMEOUT (include/vp8g.h)
    assert int(mode) & vp8g.MODE_QUAD, r.stdout
    assert float(secs) < 10.0, r.stdout


def test_chain_output_base_not_16b_aligned(vp8g):
    """The output base handed to vp8g_decode_batch_device 8 bytes past an aligned allocation, with
    whole-piece descriptors (offsets and strides 16-B aligned): the quad chain must not take its
    paired-store instantiation (which assumes a 16-B aligned base) -- and the pairs chain
    (VP8G_QUAD=0) must be exact too; every slot equals the oracle's output and the 8 bytes before
    the base stay untouched."""
    code = r"""
import ctypes as C, sys
sys.path.insert(0, sys.argv[1] + "/webp-decoder_amd")
import numpy as np, torch, vp8g, vp8g_batch
dev = torch.device("cuda:0")
n = 2 * torch.cuda.get_device_properties(0).multi_processor_count
frames = [vp8g.synth_frame(160, 64, 0xA11 ^ i, profile=i % 3) for i in range(8)]
b = vp8g_batch.DeviceBatch(n, 160, 64, dev)
for i in range(n):
    b.fill(i, frames[i % 8], i % 3 != 0)
b.commit()
big = torch.full((n * b.frame_bytes + 64,), 0xA5, dtype=torch.uint8, device=dev)
lib = vp8g.gpu_lib()
stream = torch.cuda.current_stream(dev).cuda_stream
rc = lib.vp8g_decode_batch_device(b.h_descs, C.c_void_p(b.d_descs.data_ptr()), n, C.byref(b.c_arrays),
                                  C.c_void_p(big.data_ptr() + 8), C.c_void_p(stream), 0)
assert rc == 0, lib.vp8g_last_error()
torch.cuda.synchronize()
host = big.cpu().numpy()
exp, bad = {}, []
for i in range(n):
    key = (i % 8, i % 3 != 0)
    if key not in exp:
        exp[key] = vp8g.oracle_reconstruct(frames[i % 8], key[1])
    o = 8 + i * b.frame_bytes
    if host[o:o + len(exp[key])].tobytes() != exp[key]:
        bad.append(i)
if host[:8].tobytes() != b"\xa5" * 8:
    bad.append("bytes before the base written")
print(b.launch_mode(), "OK" if not bad and b.status_word() == 0 else f"BAD {bad[:8]} status {b.status_word()}")
"""
    for env_extra in ({}, {"VP8G_QUAD": "0"}):
        env = dict(os.environ, **env_extra)
        r = subprocess.run([sys.executable, "-c", code, str(ROOT)], capture_output=True, text=True, timeout=240, env=env)
        assert r.returncode == 0, (env_extra, r.stderr[-2000:])
        assert r.stdout.strip().endswith("OK"), (env_extra, r.stdout)
        mode = int(r.stdout.split()[-2])
        assert mode & vp8g.MODE_CHAIN and bool(mode & vp8g.MODE_QUAD) == (not env_extra), (env_extra, mode)
