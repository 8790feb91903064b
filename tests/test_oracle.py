"""CPU tests: the oracle (our C restatement of m06/m07) and the host front end, pinned against the
golden manifests generated from the reference itself (tests/golden/make_manifest.py).

These establish that the checker used by the GPU tests is right:
  * every fixture: front-end coefficient hash == reference hash; oracle -yuv/-yuvf sha256 ==
    reference decoder output (which also equals libwebp's, per the manifest);
  * seeded synthetic frames (incl. stress profiles) == reference m06/m07 hashes;
  * where the reference build is present (this container): array-for-array equality of the
    front end with the reference m05, and of the loop filter alone.
"""
import ctypes as C
import hashlib

import numpy as np
import pytest

from conftest import FIXTURES


def sha(b):
    return hashlib.sha256(b).hexdigest()


def test_manifest_covers_reference_corpus(manifest):
    # the reference m6/m7 gate glob (scripts/m7_compare_yuv_filtered_with_oracle.sh:29) = 429 files,
    # plus the 4 penguins and our 10 large libwebp-encoded frames
    files = manifest["files"]
    assert sum(1 for k in files if k.split("/")[0] in ("webp", "testimages", "generated")) == 429
    assert sum(1 for k in files if k.startswith("commons/")) == 4
    assert sum(1 for k in files if k.startswith("big/")) == 10
    assert manifest["libwebp_agreement"] == {"yuv": "443/443", "yuvf": "443/443", "rgb": "443/443", "png_out": "90/90"}


def test_oracle_and_front_end_vs_manifest(vp8g, manifest):
    bad = []
    for rel, ent in sorted(manifest["files"].items()):
        f = vp8g.decode_file(FIXTURES / rel)
        if "0x%016x" % f.frame.stats.coeff_hash_fnv1a64 != ent["coeff_hash"]:
            bad.append((rel, "coeff_hash"))
        assert (f.width, f.height) == (ent["width"], ent["height"])
        for filt, key in ((False, "yuv_sha256"), (True, "yuvf_sha256")):
            if sha(vp8g.oracle_reconstruct(f, filt)) != ent[key]:
                bad.append((rel, key))
        f.free()
    assert not bad, bad[:10]


def test_oracle_ppm_png_vs_manifest(vp8g, manifest):
    """m08/m09 restatement (YUV->RGB fancy upsampling, PPM and PNG writers) vs sha256 of the
    reference decoder's own -ppm / -png files on every fixture (manifest: those equal libwebp's RGB
    on all 441 files and the pixels of the reference's 90 dwebp PNG goldens)."""
    bad = []
    for rel, ent in sorted(manifest["files"].items()):
        f = vp8g.decode_file(FIXTURES / rel)
        i420 = vp8g.oracle_reconstruct(f, True)
        for fmt in ("ppm", "png"):
            if sha(vp8g.oracle_encode(i420, f.width, f.height, fmt)) != ent[fmt + "_sha256"]:
                bad.append((rel, fmt))
        f.free()
    assert not bad, bad[:10]


def test_oracle_vs_synth_kat(vp8g, synth_kat):
    for case in synth_kat["cases"]:
        f = vp8g.synth_frame(case["width"], case["height"], case["seed"], case["profile"])
        assert sha(vp8g.oracle_reconstruct(f, False)) == case["yuv_sha256"], case
        assert sha(vp8g.oracle_reconstruct(f, True)) == case["yuvf_sha256"], case
        f.free()


def test_synth_generator_is_deterministic(vp8g):
    a = vp8g.synth_frame(129, 77, 42, 1)
    b = vp8g.synth_frame(129, 77, 42, 1)
    for name, _, _ in vp8g.FRAME_ARRAYS:
        assert np.array_equal(a.array(name), b.array(name)), name
    c = vp8g.synth_frame(129, 77, 43, 1)
    assert not np.array_equal(a.array("coeff_y"), c.array("coeff_y"))


needs_ref = pytest.mark.skipif("not __import__('vp8g').ref_available()", reason="reference build absent")


@needs_ref
def test_front_end_matches_reference_m05(vp8g, manifest):
    lib = vp8g.ref_lib()
    for rel in sorted(manifest["files"])[::7]:
        p = FIXTURES / rel
        ours = vp8g.decode_file(p)
        kf, fr = vp8g.Vp8KeyFrameHeader(), vp8g.Vp8DecodedFrame()
        assert lib.ref_decode_frame(str(p).encode(), C.byref(kf), C.byref(fr)) == 0
        theirs = vp8g.Frame(kf, fr)
        theirs._alive = False
        assert bytes(ours.kf) == bytes(kf)
        for name, _, _ in vp8g.FRAME_ARRAYS:
            assert np.array_equal(ours.array(name), theirs.array(name)), (rel, name)
        assert bytes(ours.frame)[:40] == bytes(fr)[:40]
        assert bytes(ours.frame.stats) == bytes(fr.stats), rel
        lib.ref_free_frame(C.byref(fr))
        ours.free()


@needs_ref
@pytest.mark.parametrize("seed,profile", [(1, 0), (2, 1), (3, 2), (4, 1)])
def test_oracle_loopfilter_alone_matches_reference(vp8g, seed, profile):
    f = vp8g.synth_frame(200, 130, seed, profile)
    w, h = int(f.frame.mb_cols) * 16, int(f.frame.mb_rows) * 16
    rng = np.random.default_rng(seed)
    planes = [rng.integers(0, 256, size=n, dtype=np.uint8) for n in (w * h, w * h // 4, w * h // 4)]
    ours = [p.copy() for p in planes]
    ref = [p.copy() for p in planes]
    assert vp8g.oracle_lib().oracle_loopfilter(*[p.ctypes.data for p in ours], C.byref(f.frame)) == 0
    assert vp8g.ref_lib().ref_loopfilter_padded(*[p.ctypes.data for p in ref], w, h, C.byref(f.frame)) == 0
    for a, b in zip(ours, ref):
        assert np.array_equal(a, b)


@needs_ref
@pytest.mark.parametrize("w,h,profile", [(1, 1, 1), (35, 19, 2), (333, 97, 1), (640, 360, 0), (801, 67, 2)])
def test_oracle_vs_reference_random_sizes(vp8g, w, h, profile):
    for seed in range(3):
        f = vp8g.synth_frame(w, h, 1000 * seed + w, profile)
        for filt in (False, True):
            assert vp8g.oracle_reconstruct(f, filt) == vp8g.ref_reconstruct(f, filt)
