"""GPU: the device batch API exactly as bench.py times it (vp8g_decode_batch_device on
caller-owned device buffers, then vp8g_frame_digests), every slot checked against the digest of the
reference decoder's own I420 (tests/golden/digests.json).

* 260 x 4K (> 256 CUs: the timed chain kernel `frame_kernel<16, false, false, true>` with the
  mirror split, two frames per workgroup at most);
* 512 x 4K: the exact uhd4 launch bench.py times (rank 0's shard of BASELINE configs[3] / [4]);
* 128 synthetic 4K frames of a far shard (global indices 3584..3711: rank 7 of configs[4]);
* two threads on two streams issuing 300-frame 4K batches back to back while a third calls the
  single-frame drop-in entry point: the process-wide launch gate (vp8g_device.h, GateScope) keeps
  the cross-workgroup launch modes from running beside another launch;
* 1100 x 1080p (the fhd4 workload's geometry);
* 300 mixed 4K / 1080p frames in a scrambled order (the cost-balanced launch order);
* 64 distinct synthetic 4K frames of the bench's synthetic batch (seed 0x5EED ^ i);
* the digest kernel against the numpy restatement on odd sizes (tail words, unaligned lengths);
* a stalled producer (test build lib/diag/libvp8g_stall.so: one wave never publishes, waits give
  up after 20 ms) ends the call promptly with EIO instead of waiting once per step;
* the chain with ~7 mixed small frames per workgroup, and the same forced into the mirror split.
Reference path: src/m06_recon/vp8_recon.c:718 (vp8_reconstruct_keyframe_yuv_filtered).
"""
import ctypes as C
import json
import subprocess
import sys
import time

import numpy as np
import pytest
import torch

from conftest import FIXTURES, GOLDEN, ROOT

pytestmark = pytest.mark.gpu

UHD = ["big/uhd_a_normal_seg4.webp", "big/uhd_b_simple_sharp3.webp", "big/uhd_c_normal_sharp6_seg1.webp",
       "big/uhd_d_normal_q90.webp"]
FHD = ["big/fhd_normal_sharp5.webp", "big/fhd_simple_sharp3.webp", "big/fhd_c_normal_q85_seg4.webp",
       "big/fhd_d_normal_sharp2_seg1.webp"]


@pytest.fixture(scope="module")
def digests():
    return json.loads((GOLDEN / "digests.json").read_text())


def run_batch(vp8g, rels, n, filtered, digests, slot0=0):
    import vp8g_batch
    dev = torch.device("cuda:0")
    frames = [vp8g.decode_file(FIXTURES / r) for r in rels]
    b = vp8g_batch.DeviceBatch(n, frames[0].width, frames[0].height, dev)
    b.replicate(frames, filtered, slot0=slot0)
    b.commit()
    stream = torch.cuda.current_stream(dev).cuda_stream
    b.launch(stream)
    torch.cuda.synchronize()
    assert b.status_word() == 0
    got = b.digests(stream)
    key = "yuvf" if filtered else "yuv"
    exp = [int(digests["fixtures"][rels[(slot0 + i) % len(rels)]][key], 16) for i in range(n)]
    bad = [i for i in range(n) if int(got[i]) != exp[i]]
    for f in frames:
        f.free()
    return b, bad


@pytest.mark.parametrize("filtered", [True, False], ids=["yuvf", "yuv"])
def test_device_batch_260_uhd_every_slot(vp8g, digests, filtered):
    b, bad = run_batch(vp8g, UHD, 260, filtered, digests, slot0=1)
    assert not bad, f"{len(bad)} of 260 slots differ, e.g. {bad[:8]}"
    # the digest kernel agrees with the numpy restatement on whole outputs too
    for i in (0, 259):
        assert vp8g.digest64(b.frame_output(i)) == int(b.digests(torch.cuda.current_stream().cuda_stream)[i])
    del b
    torch.cuda.empty_cache()


def test_device_batch_1100_fhd_every_slot(vp8g, digests):
    b, bad = run_batch(vp8g, FHD, 1100, True, digests)
    assert not bad, f"{len(bad)} of 1100 slots differ, e.g. {bad[:8]}"
    del b
    torch.cuda.empty_cache()


def test_device_batch_mixed_sizes_launch_order(vp8g, digests):
    """300 slots mixing 4K and 1080p frames of all eight filter setups in a scrambled order: more
    frames than CUs and differing cost classes, so the kernel runs under the cost-balanced launch
    order (workgroup -> frame by the in-kernel histogram + ballot scan, csrc/vp8g_device.h
    cost_class); every slot must still hold its own frame's reference output."""
    import vp8g_batch
    rels = UHD + FHD
    frames = [vp8g.decode_file(FIXTURES / r) for r in rels]
    n = 300
    rng = np.random.default_rng(7)
    pick = rng.integers(0, len(rels), n)
    b = vp8g_batch.DeviceBatch(n, 3840, 2160, torch.device("cuda:0"))
    for i, j in enumerate(pick):
        b.place(i, frames[j], True)
    b.commit()
    stream = torch.cuda.current_stream().cuda_stream
    b.launch(stream)
    got = b.digests(stream)
    assert b.status_word() == 0
    exp = [int(digests["fixtures"][rels[j]]["yuvf"], 16) for j in pick]
    bad = [i for i in range(n) if int(got[i]) != exp[i]]
    assert not bad, f"{len(bad)} of {n} slots differ, e.g. {bad[:8]}"
    for f in frames:
        f.free()
    del b
    torch.cuda.empty_cache()


def test_device_batch_synthetic_distinct_frames(vp8g, digests):
    import vp8g_batch
    s = digests["synth_uhd"]
    n = 64
    b = vp8g_batch.DeviceBatch(n, s["width"], s["height"], torch.device("cuda:0"))
    for i in range(n):
        f = vp8g.synth_frame(s["width"], s["height"], 0x5EED ^ i, s["profile"])
        b.fill(i, f, True)
        f.free()
    b.commit()
    stream = torch.cuda.current_stream().cuda_stream
    b.launch(stream)
    got = b.digests(stream)
    assert b.status_word() == 0
    assert [("0x%016x" % int(d)) for d in got] == s["yuvf"][:n]
    del b
    torch.cuda.empty_cache()


@pytest.mark.parametrize("w,h", [(333, 197), (17, 9), (1, 1), (1917, 1083)])
def test_digest_kernel_vs_restatement_odd_sizes(vp8g, w, h):
    import vp8g_batch
    n = 5
    b = vp8g_batch.DeviceBatch(n, w, h, torch.device("cuda:0"))
    frames = [vp8g.synth_frame(w, h, 77 * i + w, 1) for i in range(n)]
    for i, f in enumerate(frames):
        b.fill(i, f, True)
    b.commit()
    stream = torch.cuda.current_stream().cuda_stream
    b.launch(stream)
    got = b.digests(stream)
    for i, f in enumerate(frames):
        out = b.frame_output(i)
        assert out == vp8g.oracle_reconstruct(f, True), (w, h, i)
        assert int(got[i]) == vp8g.digest64(out), (w, h, i)
        f.free()


def test_stalled_producer_ends_promptly_with_eio(vp8g):
    """a timed-out dependency wait is sticky, so a producer that never publishes costs
    one wait bound per waiting wave, not one per step (the 4K frame has 242 steps per pair)."""
    code = r"""
import ctypes as C, sys, time
sys.path.insert(0, sys.argv[1] + "/webp-decoder_amd")
import vp8g
vp8g._libs["gpu"] = C.CDLL(sys.argv[1] + "/webp-decoder_amd/lib/diag/libvp8g_stall.so", use_errno=True)
f = vp8g.decode_file(sys.argv[1] + "/tests/fixtures/big/uhd_a_normal_seg4.webp")
lib = vp8g.gpu_lib()
img = vp8g.Yuv420Image()
t = time.time()
rc = lib.vp8_reconstruct_keyframe_yuv_filtered(C.byref(f.kf), C.byref(f.frame), C.byref(img))
print(rc, C.get_errno(), round(time.time() - t, 3), lib.vp8g_last_error().decode())
"""
    r = subprocess.run([sys.executable, "-c", code, str(ROOT)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    rc, err, secs, *msg = r.stdout.split()
    assert int(rc) == -1 and int(err) == 5, r.stdout  # EIO
    assert "status" in " ".join(msg)
    assert float(secs) < 10.0, r.stdout


def test_chain_many_small_mixed_frames_and_empty_slots(vp8g):
    """Chain mode (vp8g_kernels.hip: one 16-wave workgroup per CU decodes a cost-sorted list of
    frames as one chain of MB row pairs, two LDS context slots reused every other frame): 1 800
    slots, ~7 frames per workgroup, of 48 distinct synthetic frames from 1x1 to 160x96 -- single-MB
    and single-row frames (a pair of one row), odd sizes, all synthetic profiles (segments,
    loop-filter deltas, simple and normal filter, +-2114 coefficients) -- in a scrambled order with
    one slot in eight left empty (an all-zero descriptor: no work).  Every decoded slot must equal
    the oracle's output for its frame and the empty slots' outputs must stay untouched."""
    import vp8g_batch
    dev = torch.device("cuda:0")
    rng = np.random.default_rng(11)
    # (the two wide frames make the context slots large enough for the in-kernel cost sort)
    sizes = [(1, 1), (16, 16), (17, 9), (160, 16), (33, 47), (160, 96), (1024, 16), (8, 96), (1000, 40)]
    frames = []
    for i in range(48):
        w, h = sizes[i % len(sizes)]
        frames.append(vp8g.synth_frame(w, h, 0xC4A1 ^ i, profile=i % 3))
    n = 1800
    b = vp8g_batch.DeviceBatch(n, 1024, 96, dev)
    b.out.fill_(0xA5)
    pick = rng.integers(0, len(frames), n)
    empty = set(rng.choice(n, n // 8, replace=False).tolist())
    for i in range(n):
        if i not in empty:
            b.place(i, frames[pick[i]], bool(pick[i] % 2))
    b.commit()
    stream = torch.cuda.current_stream(dev).cuda_stream
    b.launch(stream)
    torch.cuda.synchronize()
    assert b.status_word() == 0
    exp = {}
    bad = []
    for i in range(n):
        if i in empty:
            continue
        j = int(pick[i])
        key = (j, bool(j % 2))
        if key not in exp:
            exp[key] = vp8g.oracle_reconstruct(frames[j], bool(j % 2))
        got = b.frame_output(i)[:len(exp[key])]
        if got != exp[key]:
            bad.append(i)
    assert not bad, f"{len(bad)} of {n - len(empty)} slots differ, e.g. {bad[:8]}"
    for i in sorted(empty)[:16]:
        assert b.frame_output(i) == b"\xa5" * b.i420, i
    for f in frames:
        f.free()


def test_chain_mirror_split_forced(vp8g):
    """Mirror split of the chain (vp8g_kernels.hip, kSegTop: a frame's top half decoded first by its
    own workgroup, its bottom half last by the mirror workgroup from a context snapshot), forced on
    for a batch of ~6 mixed small frames per workgroup (VP8G_SPLITCHAIN=1, tests/chain_split_check.py
    in a child process), two launches (the flags' epoch advances), every slot against the oracle.
    The bench's uhd4 batch takes the split by default (two 4K frames per CU): 260 x 4K above."""
    import os
    env = dict(os.environ, VP8G_SPLITCHAIN="1")
    r = subprocess.run([sys.executable, str(ROOT / "tests" / "chain_split_check.py")], capture_output=True, text=True,
                       timeout=240, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    assert r.stdout.strip().endswith("OK"), r.stdout


def test_device_batch_512_uhd_bench_launch(vp8g, digests):
    """Verdict r03 #3: the launch bench.py times for uhd4 (512 x 4K, slot i <- fixture i % 4, rank
    0's shard of BASELINE configs[3] / [4]): the chain kernel with the mirror split, every slot."""
    b, bad = run_batch(vp8g, UHD, 512, True, digests, slot0=0)
    assert not bad, f"{len(bad)} of 512 slots differ, e.g. {bad[:8]}"
    mode = b.launch_mode()  # (the quad chain, as bench.py's launch)
    assert mode & vp8g.MODE_CHAIN and mode & vp8g.MODE_QUAD, mode
    # (the mirror split needs at most two frames per workgroup: 512 frames on >= 256 CUs, as on
    # MI355X; a part with fewer CUs decodes the same batch without it -- ADVICE r05)
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    if -(-512 // cus) <= 2:
        assert mode & vp8g.MODE_MIRROR_SPLIT, mode
    del b
    torch.cuda.empty_cache()


def test_device_batch_synthetic_far_shard(vp8g, digests):
    """Verdict r03 #3: frames no other test decodes on hardware -- global indices 3584..3711 of the
    synthetic batch (seed 0x5EED ^ i; rank 7's shard of BASELINE configs[4]), against the digests of
    the reference decoder's own output (tests/golden/make_digests.py)."""
    import concurrent.futures as cf
    import vp8g_batch
    s = digests["synth_uhd"]
    lo, hi = 3584, 3712
    assert len(s["yuvf"]) >= hi
    n = hi - lo
    b = vp8g_batch.DeviceBatch(n, s["width"], s["height"], torch.device("cuda:0"))
    with cf.ThreadPoolExecutor(8) as ex:
        for i, f in enumerate(ex.map(lambda g: vp8g.synth_frame(s["width"], s["height"], 0x5EED ^ g, s["profile"]), range(lo, hi))):
            b.fill(i, f, True)
            f.free()
    b.commit()
    stream = torch.cuda.current_stream().cuda_stream
    b.launch(stream)
    got = b.digests(stream)
    assert b.status_word() == 0
    assert [("0x%016x" % int(d)) for d in got] == s["yuvf"][lo:hi]
    del b
    torch.cuda.empty_cache()


def test_device_batches_two_streams_and_dropin_concurrently(vp8g, digests):
    """Verdict r03 #2 / ADVICE r03 (medium): vp8g_decode_batch_device returns before its kernel ends,
    so two callers on two streams can have launches in flight at once.  300 x 4K per caller takes the
    chain's mirror split when alone (bottom segments wait on another workgroup's top segment); two
    such launches side by side, or one beside another kernel, could leave workgroups spinning on
    partners that cannot get a CU.  Two threads issue four launches each on their own streams while
    the main thread makes single-frame drop-in calls (whose split mode waits across workgroups too):
    every status word must stay 0 and every slot and drop-in output must match the reference."""
    import threading
    import vp8g_batch
    dev = torch.device("cuda:0")
    frames = [vp8g.decode_file(FIXTURES / r) for r in UHD]
    batches, streams = [], []
    for t in range(2):
        b = vp8g_batch.DeviceBatch(300, 3840, 2160, dev)
        b.replicate(frames, True, slot0=1 + t)
        b.commit()
        batches.append(b)
        streams.append(torch.cuda.Stream(dev))
    torch.cuda.synchronize()
    errs = []

    def worker(b, st):
        try:
            for _ in range(4):
                b.launch(st.cuda_stream)
        except Exception as e:  # noqa: BLE001 (reported below)
            errs.append(repr(e))

    th = [threading.Thread(target=worker, args=(b, st)) for b, st in zip(batches, streams)]
    for t in th:
        t.start()
    dropins = [vp8g.gpu_reconstruct(frames[i % 4], True) for i in range(3)]
    for t in th:
        t.join(timeout=120)
    assert not any(t.is_alive() for t in th)
    torch.cuda.synchronize()
    assert not errs, errs
    for t, b in enumerate(batches):
        assert b.status_word() == 0, f"batch {t}: status 0x{b.status_word():x}"
        got = b.digests(streams[t].cuda_stream)
        exp = [int(digests["fixtures"][UHD[(1 + t + i) % 4]]["yuvf"], 16) for i in range(300)]
        bad = [i for i in range(300) if int(got[i]) != exp[i]]
        assert not bad, f"batch {t}: {len(bad)} of 300 slots differ, e.g. {bad[:8]}"
    for i, out in enumerate(dropins):
        assert vp8g.digest64(out) == int(digests["fixtures"][UHD[i % 4]]["yuvf"], 16), i
    for f in frames:
        f.free()
    del batches
    torch.cuda.empty_cache()


@pytest.mark.parametrize("w,h", [(160, 96), (176, 80)])
def test_chain_two_frame_interleave(vp8g, w, h):
    """Two-frame interleave of the chain (vp8g_kernels.hip: a workgroup's frames run two at a time with
    their MB row pairs alternating, four LDS context slots; chosen for batches of one frame size with at
    least two frames per workgroup, pick_chain_interleave): 549 distinct synthetic frames, so workgroups
    hold two or three frames (an odd last frame runs alone); 176x80 has an odd MB row count (the last
    pair of every frame is a single row).  Every slot against the oracle; the launch mode read back
    (vp8g_last_launch_mode) must be the interleaved chain."""
    import vp8g_batch
    dev = torch.device("cuda:0")
    # (two frames per workgroup and, for every seventh, a third: derived from the CU count, so the
    # interleave -- it needs at least two frames per workgroup -- is chosen on any part)
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    n = 2 * cus + cus // 7
    b = vp8g_batch.DeviceBatch(n, w, h, dev)
    frames = [vp8g.synth_frame(w, h, 0x1A7E ^ i, profile=i % 3) for i in range(n)]
    for i, f in enumerate(frames):
        b.fill(i, f, bool(i % 5))
    b.commit()
    stream = torch.cuda.current_stream(dev).cuda_stream
    b.launch(stream)
    torch.cuda.synchronize()
    assert b.status_word() == 0
    mode = b.launch_mode()
    assert mode & vp8g.MODE_CHAIN and mode & vp8g.MODE_INTERLEAVE, mode
    bad = [i for i, f in enumerate(frames) if b.frame_output(i) != vp8g.oracle_reconstruct(f, bool(i % 5))]
    assert not bad, f"{len(bad)} of {n} slots differ, e.g. {bad[:8]}"
    for f in frames:
        f.free()
