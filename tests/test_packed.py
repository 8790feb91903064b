"""CPU tests of the packed m05 wire format (include/vp8g.h Vp8gPackedFrame), the
input of the end-to-end batch path (vp8g_decode_webp_batch).

The packed decode runs the same m05 as the dense one (webp-decoder_amd/host/vp8_parse.c) with a
different sink, so the bar is: side arrays identical, masks + values expand (vp8g.unpack_coeffs,
the host restatement of the device expand_kernel) to exactly the dense arrays, and with
VP8F_PACK_HASH the FNV-1a coefficient hash equals the reference's (`decoder -info`,
vp8_tokens.c:970-998; tests/golden/manifest.json "coeff_hash").
"""
import numpy as np
import pytest

from conftest import FIXTURES, ROOT

SIDE = ("ymode", "uv_mode", "segment_id", "has_coeff", "bmode", "skip_coeff")


def packed_matches_dense(vp8g, rel):
    data = (FIXTURES / rel).read_bytes()
    pf = vp8g.PackedFrame(data)
    f = vp8g.decode_file(FIXTURES / rel)
    try:
        assert (pf.p.kf.width, pf.p.kf.height) == (f.width, f.height)
        for k in SIDE:
            assert np.array_equal(pf.side(k), f.array(k)), (rel, k)
        dense = vp8g.unpack_coeffs(pf)
        for k, v in dense.items():
            assert np.array_equal(v, f.array(k)), (rel, k)
        # masks say exactly where the non-zeros are; mb_off is the running value count
        m = pf.masks()
        cnt = np.array([bin(int(x)).count("1") for x in m.reshape(-1)]).reshape(m.shape).sum(axis=1)
        assert np.array_equal(pf.mb_off(), np.concatenate([[0], np.cumsum(cnt)[:-1]]).astype(np.uint32))
        assert int(pf.p.n_values) == int(cnt.sum())
        assert not np.any(pf.values() == 0)
    finally:
        pf.free()
        f.free()


def test_packed_equals_dense_on_corpus_sample(vp8g, manifest):
    rels = sorted(manifest["files"])
    for rel in rels[::7] + ["big/fhd_simple_sharp3.webp", "commons/penguin-q80.webp"]:
        packed_matches_dense(vp8g, rel)


def test_packed_equals_dense_4k(vp8g):
    packed_matches_dense(vp8g, "big/uhd_d_normal_q90.webp")


def test_packed_hash_equals_reference(vp8g, manifest):
    for rel in sorted(manifest["files"])[::23]:
        pf = vp8g.PackedFrame((FIXTURES / rel).read_bytes(), hash_coeffs=True)
        assert "0x%016x" % pf.p.f.stats.coeff_hash_fnv1a64 == manifest["files"][rel]["coeff_hash"], rel
        pf.free()
        pf = vp8g.PackedFrame((FIXTURES / rel).read_bytes())
        assert pf.p.f.stats.coeff_hash_fnv1a64 == 0  # hashing is opt-in on the packed path
        pf.free()


@pytest.mark.parametrize("name,stage", [("empty_riff.webp", 2), ("truncated.webp", 2)])
def test_packed_errors(vp8g, name, stage):
    import ctypes as C
    data = (ROOT / "tests" / "fixtures_err" / name).read_bytes()
    p, st = vp8g.Vp8gPackedFrame(), C.c_int(0)
    buf = (C.c_uint8 * max(1, len(data))).from_buffer_copy(data or b"\0")
    assert vp8g.host_lib().vp8f_decode_packed_memory(buf, len(data), C.byref(p), C.byref(st), 0) == -1
    assert st.value >= stage
    assert not p.masks and not p.values and not p.f.ymode  # nothing leaked / left allocated


def truncated_payload(data: bytes, frac: float) -> bytes:
    """The same .webp with its VP8 payload cut to `frac` (container sizes rewritten), so the token
    partition runs past its end and the bool decoder's overread diagnostics come into play."""
    import struct
    csize = struct.unpack("<I", data[16:20])[0]
    c = int(csize * frac)
    c -= c & 1
    return b"RIFF" + struct.pack("<I", 12 + c) + b"WEBPVP8 " + struct.pack("<I", c) + data[20:20 + c]


@pytest.mark.skipif(not (ROOT / "oracle" / "_ref" / "libref.so").exists(), reason="reference not built here")
def test_front_end_stats_equal_reference_on_truncated_streams(vp8g, manifest, tmp_path):
    """m05 statistics (Vp8CoeffStats: counts, hash, bytes used, first overread position and stage,
    vp8_tokens.c:970-998 and bool_decoder.c:5-39) of the host front end -- dense and packed -- equal the
    reference's own m05 (oracle/_ref/libref.so) on intact and truncated payloads."""
    import ctypes as C
    ref = vp8g.ref_lib()
    host = vp8g.host_lib()
    n_ovr = 0
    for rel in sorted(manifest["files"])[::9]:
        data = (FIXTURES / rel).read_bytes()
        for frac in (1.0, 0.95, 0.8):
            case = data if frac == 1.0 else truncated_payload(data, frac)
            path = tmp_path / "case.webp"
            path.write_bytes(case)
            kf, rf = vp8g.Vp8KeyFrameHeader(), vp8g.Vp8DecodedFrame()
            rrc = ref.ref_decode_frame(str(path).encode(), C.byref(kf), C.byref(rf))
            kf2, df, st = vp8g.Vp8KeyFrameHeader(), vp8g.Vp8DecodedFrame(), C.c_int(0)
            buf = (C.c_uint8 * len(case)).from_buffer_copy(case)
            drc = host.vp8f_decode_memory(buf, len(case), C.byref(kf2), C.byref(df), C.byref(st))
            assert (rrc == 0) == (drc == 0), (rel, frac)
            if rrc == 0:
                assert bytes(df.stats) == bytes(rf.stats), (rel, frac)
                n_ovr += rf.stats.token_overread
                pf = vp8g.PackedFrame(case, hash_coeffs=True)
                assert bytes(pf.p.f.stats) == bytes(rf.stats), (rel, frac, "packed")
                pf.free()
                ref.ref_free_frame(C.byref(rf))
                host.vp8_decoded_frame_free(C.byref(df))
    assert n_ovr > 10  # the truncations did reach the overread paths


def test_token_header_matches_front_end(vp8g, manifest):
    """vp8f_token_header_memory (host half of the device m05): the frame-level fields equal the
    full front end's, the job locates the partitions inside the VP8 payload and starts partition 0's
    bool decoder in a valid state."""
    import ctypes as C
    import struct
    host = vp8g.host_lib()
    hdr_fields = [n for n, _ in vp8g.Vp8DecodedFrame._fields_ if not n.startswith(("segment_id", "skip", "has_",
                  "ymode", "uv_mode", "bmode", "coeff", "stats"))]
    for rel in sorted(manifest["files"])[::3]:
        data = (FIXTURES / rel).read_bytes()
        kf, hdr, tf, off, size = vp8g.token_header(data)
        assert off == 20 and size == struct.unpack("<I", data[16:20])[0]
        kf2, df, st = vp8g.Vp8KeyFrameHeader(), vp8g.Vp8DecodedFrame(), C.c_int(0)
        buf = (C.c_uint8 * len(data)).from_buffer_copy(data)
        assert host.vp8f_decode_memory(buf, len(data), C.byref(kf2), C.byref(df), C.byref(st)) == 0
        try:
            assert bytes(kf) == bytes(kf2)
            for n in hdr_fields:
                a, b = getattr(hdr, n), getattr(df, n)
                assert (list(a) if hasattr(a, "__len__") else a) == (list(b) if hasattr(b, "__len__") else b), (rel, n)
            assert (tf.mb_cols, tf.mb_rows) == (df.mb_cols, df.mb_rows)
            assert tf.p0_end == 10 + kf.first_partition_len == tf.tok_off and tf.tok_end == size
            assert 128 <= tf.b_range <= 255 and 0 <= tf.b_bits <= 56 and 10 < tf.b_next <= tf.p0_end
            assert tf.seg_enabled == df.segmentation_enabled
            probs = np.frombuffer(bytes(tf.coeff_probs), np.uint8).reshape(4, 8, 3, 12)
            assert (probs[..., 11] == 0).all()  # the pad byte of each 12-byte row
        finally:
            host.vp8_decoded_frame_free(C.byref(df))


def test_token_header_rejects(vp8g):
    for name in ("empty_riff.webp", "truncated.webp"):
        with pytest.raises(ValueError):
            vp8g.token_header((ROOT / "tests" / "fixtures_err" / name).read_bytes())
    with pytest.raises(ValueError):
        vp8g.token_header(b"")
