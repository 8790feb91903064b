"""CPU checks of the parity digests and the golden files the GPU runs compare against.

* vp8g.digest64 (numpy) equals a plain-Python loop over the definition in include/vp8g.h
  (vp8g_frame_digests), on lengths around every word / chunk boundary;
* tests/golden/digests.json (digests of the reference decoder's own I420) is reproduced by our
  oracle restatement for every bench fixture and for sampled synthetic frames of the bench's
  synthetic batch (seed 0x5EED ^ i, vp8_synth.c profile 0);
* tests/golden/multipart.json (libwebp's decode of libwebp-encoded 2/4/8-partition streams, which
  the reference rejects: src/m05_tokens/vp8_tokens.c:357-360) is reproduced by the host front end's
  opt-in multi-partition decode + the oracle.
"""
import ctypes as C
import hashlib
import json

import numpy as np
import pytest

from conftest import FIXTURES, GOLDEN, ROOT

MASK = (1 << 64) - 1
K = 0x9E3779B97F4A7C15


def digest_py(b: bytes) -> int:
    def mix(z):
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & MASK
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & MASK
        return z ^ (z >> 31)
    d = len(b) * K
    for i in range(0, len(b), 8):
        w = int.from_bytes(b[i:i + 8].ljust(8, b"\0"), "little")
        d += mix((w + (i // 8 + 1) * K) & MASK)
    return d & MASK


@pytest.fixture(scope="module")
def digests():
    return json.loads((GOLDEN / "digests.json").read_text())


def test_digest_numpy_equals_definition(vp8g):
    rng = np.random.default_rng(5)
    for n in (0, 1, 7, 8, 9, 15, 16, 17, 63, 64, 65, 1000, 4097):
        b = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        assert vp8g.digest64(b) == digest_py(b), n
    # order-sensitive, length-sensitive
    assert vp8g.digest64(b"\1\2") != vp8g.digest64(b"\2\1")
    assert vp8g.digest64(b"\0") != vp8g.digest64(b"\0\0")


def test_golden_fixture_digests_match_oracle(vp8g, digests, manifest):
    for rel, ent in digests["fixtures"].items():
        f = vp8g.decode_file(FIXTURES / rel)
        for filtered, key in ((False, "yuv"), (True, "yuvf")):
            out = vp8g.oracle_reconstruct(f, filtered)
            assert hashlib.sha256(out).hexdigest() == manifest["files"][rel][key + "_sha256"]
            assert "0x%016x" % vp8g.digest64(out) == ent[key], (rel, key)
        f.free()


@pytest.mark.parametrize("i", [0, 1, 511, 512, 4095])
def test_golden_synth_digests_match_oracle(vp8g, digests, i):
    s = digests["synth_uhd"]
    f = vp8g.synth_frame(s["width"], s["height"], 0x5EED ^ i, s["profile"])
    assert "0x%016x" % vp8g.digest64(vp8g.oracle_reconstruct(f, True)) == s["yuvf"][i]
    f.free()


def packed_to_i420(vp8g, data: bytes, filtered: bool) -> bytes:
    """Host multi-partition decode (packed) -> dense arrays -> oracle restatement of m06/m07."""
    p = vp8g.PackedFrame(data, multi_partition=True)
    dense = vp8g.unpack_coeffs(p)
    fr = vp8g.Vp8DecodedFrame.from_buffer_copy(bytes(p.p.f))
    keep = {k: np.ascontiguousarray(v) for k, v in dense.items()}
    for k, v in keep.items():
        setattr(fr, k, v.ctypes.data_as(C.POINTER(C.c_int16)))
    kf = vp8g.Vp8KeyFrameHeader.from_buffer_copy(bytes(p.p.kf))
    buf = np.empty(vp8g.i420_size(kf.width, kf.height), np.uint8)
    assert vp8g.oracle_lib().oracle_reconstruct_i420(C.byref(kf), C.byref(fr), buf.ctypes.data, int(filtered)) == 0
    p.free()
    return buf.tobytes()


def test_libwebp_multipartition_fixtures_host_decode(vp8g):
    mp = json.loads((GOLDEN / "multipart.json").read_text())
    assert sorted(e["partitions"] for e in mp["files"].values()) == [2, 2, 4, 4, 8, 8, 8]
    for name, ent in mp["files"].items():
        data = (ROOT / "tests" / "fixtures_mp" / name).read_bytes()
        with pytest.raises(ValueError):
            vp8g.PackedFrame(data)  # the reference's behaviour by default: ENOTSUP
        for filtered, key in ((False, "yuv"), (True, "yuvf")):
            out = packed_to_i420(vp8g, data, filtered)
            assert hashlib.sha256(out).hexdigest() == ent[key + "_sha256"], (name, key)
            assert "0x%016x" % vp8g.digest64(out) == ent[key + "_digest"]
