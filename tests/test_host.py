"""CPU tests: the C-ABI library surface, descriptor computation, front-end error behaviour and
the CLI contract (no GPU compute is invoked here)."""
import ctypes as C
import pathlib
import re
import subprocess

import numpy as np
import pytest

from conftest import FIXTURES, ROOT

DECODER = ROOT / "webp-decoder_amd" / "bin" / "decoder"


def header_functions():
    txt = (ROOT / "include" / "vp8g.h").read_text()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:const\s+)?[A-Za-z_][\w\s\*]*?\b([a-z_][a-z0-9_]*)\s*\(", txt, flags=re.M)))


def test_header_declares_reference_entry_points():
    fns = header_functions()
    for name in ("yuv420_alloc", "yuv420_free", "vp8_reconstruct_keyframe_yuv",
                 "vp8_reconstruct_keyframe_yuv_filtered", "vp8_loopfilter_apply_keyframe"):
        assert name in fns


def test_library_exports_every_declared_symbol(vp8g):
    lib = vp8g.gpu_lib()
    missing = [f for f in header_functions() if not hasattr(lib, f)]
    assert not missing, missing
    assert lib.vp8g_abi_version() == 5


def test_struct_layouts(vp8g):
    # offsets the reference ABI fixes (verified with offsetof on the reference)
    D = vp8g.Vp8DecodedFrame
    assert (D.segment_id.offset, D.has_coeff.offset, D.ymode.offset, D.uv_mode.offset, D.bmode.offset) == (40, 56, 64, 72, 80)
    assert (D.coeff_y2.offset, D.coeff_y.offset, D.coeff_u.offset, D.coeff_v.offset, D.stats.offset) == (88, 96, 104, 112, 120)
    K = vp8g.Vp8KeyFrameHeader
    assert (K.width.offset, K.height.offset) == (20, 22)


def test_null_arguments_fail_with_einval(vp8g):
    lib = vp8g.gpu_lib()
    lib = C.CDLL(str(vp8g.LIB_DIR / "libvp8g.so"), use_errno=True)
    for fn in (lib.vp8_reconstruct_keyframe_yuv, lib.vp8_reconstruct_keyframe_yuv_filtered):
        C.set_errno(0)
        assert fn(None, None, None) == -1
        assert C.get_errno() == 22
    C.set_errno(0)
    assert lib.vp8_loopfilter_apply_keyframe(None, None) == -1 and C.get_errno() == 22
    img = vp8g.Yuv420Image()
    C.set_errno(0)
    assert lib.yuv420_alloc(C.byref(img), 0, 5) == -1 and C.get_errno() == 22


def test_segment_map_required_only_with_segmentation(vp8g):
    """Like the reference (vp8_recon.c:447, vp8_loopfilter.c:169-171): segment_id is read only when
    segmentation is enabled and mb_total is never read.  Without a GPU the accepted frame fails
    later with EIO, the rejected one up front with EINVAL."""
    lib = C.CDLL(str(vp8g.LIB_DIR / "libvp8g.so"), use_errno=True)
    f = vp8g.synth_frame(48, 32, 3, 0)  # profile 0: segmentation enabled
    seg = f.frame.segment_id
    d = vp8g.Vp8gFrameDesc()
    fr = vp8g.Vp8DecodedFrame.from_buffer_copy(bytes(f.frame))
    fr.segment_id = None
    C.set_errno(0)
    assert lib.vp8g_make_frame_desc(C.byref(f.kf), C.byref(fr), 1, 0, 0, C.byref(d)) == -1 and C.get_errno() == 22
    fr.segmentation_enabled = 0
    fr.mb_total = 12345  # never read
    assert lib.vp8g_make_frame_desc(C.byref(f.kf), C.byref(fr), 1, 0, 0, C.byref(d)) == 0
    assert bool(seg)


def test_loopfilter_size_mismatch_is_einval(vp8g):
    lib = C.CDLL(str(vp8g.LIB_DIR / "libvp8g.so"), use_errno=True)
    lib.yuv420_alloc.argtypes = [C.POINTER(vp8g.Yuv420Image), C.c_uint32, C.c_uint32]
    f = vp8g.synth_frame(48, 32, 1, 0)
    img = vp8g.Yuv420Image()
    assert lib.yuv420_alloc(C.byref(img), 47, 32) == 0  # not MB-aligned -> reference returns EINVAL
    C.set_errno(0)
    assert lib.vp8_loopfilter_apply_keyframe(C.byref(img), C.byref(f.frame)) == -1
    assert C.get_errno() == 22
    lib.yuv420_free(C.byref(img))


def test_yuv420_alloc_matches_reference_semantics(vp8g):
    lib = vp8g.gpu_lib()
    img = vp8g.Yuv420Image()
    assert lib.yuv420_alloc(C.byref(img), 7, 5) == 0
    assert (img.stride_y, img.stride_uv) == (7, 4)
    assert C.string_at(img.y, 35) == bytes(35)
    assert C.string_at(img.u, 12) == bytes([128]) * 12 and C.string_at(img.v, 12) == bytes([128]) * 12
    lib.yuv420_free(C.byref(img))
    assert not img.y


def _lf_params_reference(f, seg, bpred):
    # independent restatement of reference vp8_loopfilter.c:166-199 for the descriptor check
    d = f.frame
    lvl = d.lf_level
    if d.segmentation_enabled:
        s = d.seg_lf_level[seg]
        lvl = s if d.segmentation_abs else lvl + s
    lvl = min(max(lvl, 0), 63)
    if d.lf_delta_enabled:
        lvl += d.lf_ref_delta[0] + (d.lf_mode_delta[0] if bpred else 0)
        lvl = min(max(lvl, 0), 63)
    il = lvl
    if d.lf_sharpness:
        il >>= 2 if d.lf_sharpness > 4 else 1
        il = min(il, 9 - d.lf_sharpness)
    il = max(il, 1)
    return lvl, il, 2 if lvl >= 40 else (1 if lvl >= 15 else 0)


@pytest.mark.parametrize("seed,profile", [(s, p) for s in range(6) for p in (0, 1, 2)])
def test_frame_descriptor(vp8g, seed, profile):
    f = vp8g.synth_frame(100 + seed, 60 + seed, seed, profile)
    d = vp8g.make_desc(f, True, 12345, 4096)
    assert (d.mb_cols, d.mb_rows, d.width, d.height) == (f.frame.mb_cols, f.frame.mb_rows, f.width, f.height)
    assert d.mb_offset == 12345 and d.out_y == 4096
    assert d.out_u == 4096 + f.width * f.height
    assert d.out_v == d.out_u + ((f.width + 1) // 2) * ((f.height + 1) // 2)
    any_lf = False
    for seg in range(4):
        for bp in range(2):
            exp = _lf_params_reference(f, seg, bp)
            assert tuple(d.lf[seg][bp][:3]) == exp
            any_lf |= exp[0] != 0
    assert bool(d.flags & vp8g.VP8G_F_LOOPFILTER) == any_lf
    assert bool(d.flags & vp8g.VP8G_F_SIMPLE) == bool(f.frame.lf_use_simple)
    d0 = vp8g.make_desc(f, False, 0, 0)
    assert not (d0.flags & vp8g.VP8G_F_LOOPFILTER)


def test_front_end_rejects_bad_containers(vp8g):
    for name in ("truncated.webp", "empty_riff.webp"):
        with pytest.raises(ValueError, match="stage 2"):
            vp8g.decode_file(ROOT / "tests" / "fixtures_err" / name)
    with pytest.raises(ValueError, match="stage 1"):
        vp8g.decode_file(ROOT / "tests" / "nonexistent.webp")


def test_front_end_rejects_corrupt_header(vp8g):
    data = bytearray((FIXTURES / "webp" / sorted(p.name for p in (FIXTURES / "webp").iterdir())[0]).read_bytes())
    data[20 + 3] ^= 0xFF  # break the 9d 01 2a start code
    lib = vp8g.host_lib()
    kf, fr, st = vp8g.Vp8KeyFrameHeader(), vp8g.Vp8DecodedFrame(), C.c_int()
    buf = (C.c_uint8 * len(data)).from_buffer(data)
    assert lib.vp8f_decode_memory(C.cast(buf, C.c_void_p), len(data), C.byref(kf), C.byref(fr), C.byref(st)) == -1
    assert st.value == 3


def test_cli_usage_and_errors(tmp_path):
    r = subprocess.run([str(DECODER)], capture_output=True)
    assert r.returncode == 2 and b"Usage" in r.stderr
    r = subprocess.run([str(DECODER), "-yuv", "x.webp"], capture_output=True)
    assert r.returncode == 2
    r = subprocess.run([str(DECODER), "-bogus", "a", "b"], capture_output=True)
    assert r.returncode == 2
    r = subprocess.run([str(DECODER), "-yuvf", str(ROOT / "tests/fixtures_err/truncated.webp"), str(tmp_path / "o")],
                       capture_output=True)
    assert r.returncode == 1 and b"not a supported simple lossy WebP" in r.stderr
    r = subprocess.run([str(DECODER), "-yuv", str(tmp_path / "missing.webp"), str(tmp_path / "o")], capture_output=True)
    assert r.returncode == 1


def test_cli_info_reports_reference_hash(manifest):
    rel = "commons/penguin-q20.webp"
    r = subprocess.run([str(DECODER), "-info", str(FIXTURES / rel)], capture_output=True, text=True)
    assert r.returncode == 0
    assert manifest["files"][rel]["coeff_hash"] in r.stdout


def _raw_crc(r, data):  # CRC-32 register update without conditioning (init r, no final xor)
    import zlib
    return zlib.crc32(data, r ^ 0xFFFFFFFF) ^ 0xFFFFFFFF


def _op(cols, v):
    r = 0
    for i in range(32):
        if (v >> i) & 1:
            r ^= cols[i]
    return r


@pytest.mark.parametrize("w,h", [(1, 1), (333, 97), (21845, 2), (1024, 700)])
def test_png_descriptor_and_checksum_algebra(vp8g, w, h):
    """Host side of the device PNG writer: vp8g_make_enc_desc's layout (prefix bytes, sizes) equals
    the oracle's file, and its GF(2) CRC operators -- replayed here exactly as the finishing kernel
    combines per-task CRCs (Horner over each thread's tasks, tree, un-pad, Adler patch, init) --
    give the file's IDAT CRC and Adler-32.  No GPU involved."""
    import struct
    import zlib
    rng = np.random.default_rng(w + h)
    i420 = rng.integers(0, 256, size=w * h + 2 * ((w + 1) // 2) * ((h + 1) // 2), dtype=np.uint8).tobytes()
    png = vp8g.oracle_encode(i420, w, h, "png")
    d = vp8g.Vp8gEncDesc()
    lib = vp8g.gpu_lib()
    S = vp8g.ENC_SPAN
    G = lib.vp8g_make_enc_desc(w, h, 2, 0, 0, 0, w, (w + 1) // 2, 0, 0, C.byref(d))
    assert G == (len(png) + S - 1) // S and d.file_len == len(png) == lib.vp8g_encoded_size(2, w, h)
    assert bytes(d.prefix[:d.prefix_len]) == png[:d.prefix_len]
    E = d.zend
    # per-task raw CRCs over the task's bytes, everything outside [37, E-4) read as zero
    buf = bytearray(G * S)
    buf[37:E - 4] = png[37:E - 4]
    parts = [_raw_crc(0, bytes(buf[g * S:(g + 1) * S])) for g in range(G)]
    m = (G + 255) // 256
    pad = 256 * m - G
    ops = [list(d.crc_ops[i]) for i in range(10)]
    acc = []
    for t in range(256):
        c = 0
        for i in range(m):
            gi = t * m + i - pad
            c = _op(ops[0], c) ^ (parts[gi] if gi >= 0 else 0)
        acc.append(c)
    for lvl in range(8):
        for t in range(256 >> (lvl + 1)):
            lo, hi = t << (lvl + 1), (t << (lvl + 1)) + (1 << lvl)
            acc[lo] = _op(ops[1 + lvl], acc[lo]) ^ acc[hi]
    adler = png[E - 4:E]
    crc = (_op(ops[9], acc[0]) ^ _raw_crc(0, adler) ^ d.crc_init) ^ 0xFFFFFFFF
    assert crc == struct.unpack(">I", png[E:E + 4])[0] == zlib.crc32(png[37:E])
    raw = zlib.decompress(png[41:E])
    assert struct.unpack(">I", adler)[0] == zlib.adler32(raw)
