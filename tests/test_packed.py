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
