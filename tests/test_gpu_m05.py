"""GPU tests (MI355X) of the device m05 (webp-decoder_amd/csrc/vp8g_m05.hip):
per-macroblock modes and coefficient tokens decoded on the device, one wavefront per frame, from
the partition-0 state handed over by vp8f_token_header.

Bars: the m05 arrays are bit-exact against the host front end (host/vp8_parse.c, itself pinned to
the reference's m05 by tests/test_packed.py and tests/test_host.py) for every fixture, including
payloads cut short (the token partition then reads zeros past its end, as in the reference's
bool_decoder.c:5-15); the end-to-end batch path in device-m05 mode reproduces the reference
decoder's `-yuv` / `-yuvf` output (sha256 in tests/golden/manifest.json).
"""
import hashlib
import os

import numpy as np
import pytest

from conftest import FIXTURES, ROOT
from test_packed import truncated_payload

pytestmark = pytest.mark.gpu

NAMES = ["coeff_y", "coeff_u", "coeff_v", "coeff_y2", "ymode", "uv_mode", "segment_id", "has_coeff", "bmode"]


def sha(b):
    return hashlib.sha256(b).hexdigest()


def host_arrays(vp8g, data):
    import ctypes as C
    kf, df, st = vp8g.Vp8KeyFrameHeader(), vp8g.Vp8DecodedFrame(), C.c_int(0)
    buf = (C.c_uint8 * len(data)).from_buffer_copy(data)
    assert vp8g.host_lib().vp8f_decode_memory(buf, len(data), C.byref(kf), C.byref(df), C.byref(st)) == 0
    f = vp8g.Frame(kf, df)
    out = {k: f.array(k).copy() for k in NAMES}
    f.free()
    return out


def compare(vp8g, files, labels):
    got = vp8g.gpu_m05(files)
    for data, g, lab in zip(files, got, labels):
        want = host_arrays(vp8g, data)
        for k in NAMES:
            if not np.array_equal(g[k], want[k]):
                bad = np.flatnonzero(g[k] != want[k])
                raise AssertionError(f"{lab}: {k} differs at {bad.size} entries, first {bad[:4]}")


def test_m05_arrays_corpus(vp8g, manifest):
    rels = sorted(manifest["files"])
    compare(vp8g, [(FIXTURES / r).read_bytes() for r in rels], rels)


def test_m05_arrays_truncated(vp8g, manifest):
    rels = sorted(manifest["files"])[::5]
    files, labels = [], []
    for r in rels:
        data = (FIXTURES / r).read_bytes()
        for frac in (0.97, 0.8, 0.5):
            files.append(truncated_payload(data, frac))
            labels.append(f"{r}@{frac}")
    # keep the cases whose frame header (first partition) survives the cut
    keep = []
    for f, lab in zip(files, labels):
        try:
            vp8g.token_header(f)
            keep.append((f, lab))
        except ValueError:
            pass
    assert len(keep) > 10
    compare(vp8g, [k[0] for k in keep], [k[1] for k in keep])


@pytest.mark.parametrize("filtered,key", [(True, "yuvf_sha256"), (False, "yuv_sha256")])
def test_pipeline_device_m05_corpus(vp8g, manifest, filtered, key):
    rels = sorted(manifest["files"])
    outs, st = vp8g.gpu_decode_webp_batch([(FIXTURES / r).read_bytes() for r in rels], filtered, 16, device_m05=True)
    assert st == [0] * len(rels)
    bad = [r for r, o in zip(rels, outs) if sha(o) != manifest["files"][r][key]]
    assert not bad, f"{len(bad)} mismatches, e.g. {bad[:8]}"


def test_pipeline_device_m05_chunks(vp8g, manifest, monkeypatch):
    """Several chunks (the two device slots alternate) of mixed frame sizes."""
    rels = ["big/uhd_a_normal_seg4.webp", "big/k128_normal.webp", "big/fhd_normal_sharp5.webp",
            "webp/blockcheck2_16x16_000_000_000_255_255_255_q010.webp", "commons/penguin-q20.webp"]
    files = [(FIXTURES / r).read_bytes() for r in rels]
    seq = [i % len(rels) for i in range(40)]
    monkeypatch.setenv("VP8G_CHUNK_FRAMES", "7")
    outs, st = vp8g.gpu_decode_webp_batch([files[i] for i in seq], True, 4, device_m05=True)
    assert st == [0] * len(seq)
    for i, o in zip(seq, outs):
        assert sha(o) == manifest["files"][rels[i]]["yuvf_sha256"], rels[i]


def test_pipeline_device_m05_matches_host_m05_on_truncated(vp8g, manifest):
    rels = sorted(manifest["files"])[::7]
    files = [truncated_payload((FIXTURES / r).read_bytes(), 0.7) for r in rels]
    a, sa = vp8g.gpu_decode_webp_batch(files, True, 8, device_m05=False)
    b, sb = vp8g.gpu_decode_webp_batch(files, True, 8, device_m05=True)
    assert sa == sb
    assert sum(1 for s in sa if s == 0) > 5
    assert a == b


def test_pipeline_device_m05_failed_frames_are_isolated(vp8g, manifest):
    good = ["webp/blockcheck2_16x16_000_000_000_255_255_255_q010.webp", "commons/penguin-q20.webp"]
    bad = [(ROOT / "tests" / "fixtures_err" / n).read_bytes() for n in ("empty_riff.webp", "truncated.webp")]
    files = [(FIXTURES / good[0]).read_bytes(), bad[0], b"", (FIXTURES / good[1]).read_bytes(), bad[1]]
    outs, st = vp8g.gpu_decode_webp_batch(files, True, 4, device_m05=True)
    assert st[0] == 0 and st[3] == 0 and all(s != 0 for s in (st[1], st[2], st[4]))
    assert outs[1] is None and outs[2] is None and outs[4] is None
    assert sha(outs[0]) == manifest["files"][good[0]]["yuvf_sha256"]
    assert sha(outs[3]) == manifest["files"][good[1]]["yuvf_sha256"]


@pytest.mark.parametrize("log2k", [1, 2, 3])
def test_m05_arrays_multi_partition(vp8g, manifest, log2k):
    """One token wave per partition, row wavefront between them: the m05 arrays of
    the re-partitioned frames equal the original frames' (host front end)."""
    from multipart import repartition
    rels = sorted(manifest["files"])[::3]
    orig = [(FIXTURES / r).read_bytes() for r in rels]
    got = vp8g.gpu_m05([repartition(d, log2k) for d in orig], multi_partition=True)
    for data, g, lab in zip(orig, got, rels):
        want = host_arrays(vp8g, data)
        for k in NAMES:
            assert np.array_equal(g[k], want[k]), (lab, k)


@pytest.mark.parametrize("device_m05", [False, True])
def test_pipeline_multi_partition(vp8g, manifest, device_m05):
    """Multi-partition streams end to end (opt-in) reproduce the original frames' `-yuvf` output;
    without the flag they fail like the reference (ENOTSUP) and the rest of the batch decodes."""
    from multipart import repartition
    rels = sorted(manifest["files"])[::4] + ["big/uhd_a_normal_seg4.webp", "big/uhd_d_normal_q90.webp"]
    files = [repartition((FIXTURES / r).read_bytes(), 1 + i % 3) for i, r in enumerate(rels)]
    outs, st = vp8g.gpu_decode_webp_batch(files, True, 8, device_m05=device_m05, multi_partition=True)
    assert st == [0] * len(rels)
    bad = [r for r, o in zip(rels, outs) if sha(o) != manifest["files"][r]["yuvf_sha256"]]
    assert not bad, bad[:8]
    outs, st = vp8g.gpu_decode_webp_batch(files[:3] + [(FIXTURES / rels[0]).read_bytes()], True, 4,
                                          device_m05=device_m05)
    assert all(s != 0 for s in st[:3]) and st[3] == 0


@pytest.mark.parametrize("device_m05", [False, True], ids=["host_m05", "device_m05"])
@pytest.mark.parametrize("filtered,key", [(False, "yuv"), (True, "yuvf")])
def test_libwebp_multi_partition_streams(vp8g, device_m05, filtered, key):
    """genuine 2/4/8-partition streams encoded by libwebp 1.2.2 (tests/fixtures_mp/,
    tools/make_big_fixtures.c) decode to libwebp's own I420 (tests/golden/multipart.json) in both
    batch modes; the reference rejects these streams (src/m05_tokens/vp8_tokens.c:357-360)."""
    import json
    mp = json.loads((ROOT / "tests" / "golden" / "multipart.json").read_text())
    names = sorted(mp["files"])
    files = [(ROOT / "tests" / "fixtures_mp" / n).read_bytes() for n in names]
    outs, st = vp8g.gpu_decode_webp_batch(files, filtered, 8, device_m05=device_m05, multi_partition=True)
    assert st == [0] * len(names)
    bad = [n for n, o in zip(names, outs) if sha(o) != mp["files"][n][key + "_sha256"]]
    assert not bad, bad
    gm = vp8g.gpu_m05(files, multi_partition=True)  # device m05 arrays: one token wave per partition
    for n, g in zip(names, gm):
        assert int(g["ymode"].size) == ((mp["files"][n]["width"] + 15) // 16) * ((mp["files"][n]["height"] + 15) // 16)


@pytest.mark.parametrize("hybrid", ["0", "1"], ids=["pure_device", "hybrid"])
def test_pipeline_device_m05_hybrid_split(vp8g, manifest, monkeypatch, hybrid):
    """in device-m05 mode the heaviest frames go to the host threads (packed path)
    and the rest to the device m05 (plan_frames in vp8g_pipeline.hip; VP8G_HYBRID=0 = all on the
    device).  Both schedules reproduce the reference's -yuvf output, in the callers' order."""
    monkeypatch.setenv("VP8G_HYBRID", hybrid)
    rels = ["big/uhd_d_normal_q90.webp", "big/uhd_a_normal_seg4.webp", "big/fhd_normal_sharp5.webp",
            "big/uhd_b_simple_sharp3.webp"] * 6 + sorted(manifest["files"])[::40]
    files = [(FIXTURES / r).read_bytes() for r in rels]
    outs, st = vp8g.gpu_decode_webp_batch(files, True, 4, device_m05=True)
    assert st == [0] * len(rels)
    bad = [r for r, o in zip(rels, outs) if sha(o) != manifest["files"][r]["yuvf_sha256"]]
    assert not bad, bad[:8]


def test_pipeline_hybrid_small_host_chunks_beside_device_m05(vp8g, manifest, monkeypatch):
    """host-m05 chunks of 2 frames (which alone would run in split mode) launched while
    the device-m05 chunk's long kernel runs on another stream.  Chunks of a multi-chunk call never
    split (their parts could wait on CUs another stream holds), so every frame decodes and matches
    the reference's -yuvf output."""
    monkeypatch.setenv("VP8G_HYBRID", "1")
    monkeypatch.setenv("VP8G_CHUNK_FRAMES", "2")
    rels = ["big/uhd_d_normal_q90.webp", "big/uhd_a_normal_seg4.webp", "big/fhd_normal_sharp5.webp"] * 4 + \
        sorted(manifest["files"])[::25]
    files = [(FIXTURES / r).read_bytes() for r in rels]
    outs, st = vp8g.gpu_decode_webp_batch(files, True, 4, device_m05=True)
    assert st == [0] * len(rels)
    bad = [r for r, o in zip(rels, outs) if sha(o) != manifest["files"][r]["yuvf_sha256"]]
    assert not bad, bad[:8]
