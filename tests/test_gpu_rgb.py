"""GPU parity tests (MI355X) for the m08/m09 stage: fancy-upsampled YUV->RGB and the PPM / PNG
writers on the device (libvp8g.so, webp-decoder_amd/csrc/vp8g_rgb.hip).

Bar: bit-exact files.  Pinned by the manifest's sha256 of the reference decoder's own `-ppm` /
`-png` output (equal to libwebp's RGB on all 441 fixtures and to the reference's 90 dwebp PNG
goldens, tests/golden/make_manifest.py); at other sizes by the oracle's m08/m09 restatement
(oracle/vp8_oracle.c, itself pinned by the same manifest in tests/test_oracle.py).
"""
import ctypes as C
import hashlib
import struct
import subprocess
import zlib

import numpy as np
import pytest

from conftest import FIXTURES, ROOT

pytestmark = pytest.mark.gpu


def sha(b):
    return hashlib.sha256(b).hexdigest()


def random_i420(w, h, seed):
    rng = np.random.default_rng(seed)
    n = w * h + 2 * ((w + 1) // 2) * ((h + 1) // 2)
    return rng.integers(0, 256, size=n, dtype=np.uint8).tobytes()


@pytest.mark.parametrize("fmt", ["ppm", "png"])
def test_corpus_writers_vs_manifest(vp8g, manifest, fmt):
    """yuv420_write_ppm_fd / yuv420_write_png_fd on the filtered reconstruction of every fixture
    (the reference's `decoder -ppm/-png`, src/main.c:706-844) vs the reference decoder's files."""
    bad = []
    for rel, ent in sorted(manifest["files"].items()):
        f = vp8g.decode_file(FIXTURES / rel)
        i420 = vp8g.gpu_reconstruct(f, True)
        if sha(vp8g.gpu_encode(i420, f.width, f.height, fmt)) != ent[fmt + "_sha256"]:
            bad.append(rel)
        f.free()
    assert not bad, f"{len(bad)} mismatches, e.g. {bad[:8]}"


# sizes around the layout boundaries: 1-pixel rows/columns, odd/even widths, scanlines that cross
# the 65535-byte stored-block boundary and the 32 KB task boundary, several blocks per row
SIZES = [(1, 1), (2, 1), (1, 2), (3, 3), (2, 2), (5, 7), (16, 16), (17, 1), (1, 300), (333, 97), (4000, 3),
         (21845, 2), (21844, 3), (10923, 5), (1917, 1083), (3840, 2160)]


@pytest.mark.parametrize("w,h", SIZES)
def test_random_images_vs_oracle(vp8g, w, h):
    """Random I420 planes (every chroma / luma combination the clip and upsampler can see)."""
    i420 = random_i420(w, h, w * 131 + h)
    for fmt in ("ppm", "png"):
        got = vp8g.gpu_encode(i420, w, h, fmt)
        exp = vp8g.oracle_encode(i420, w, h, fmt)
        assert len(got) == len(exp), (w, h, fmt)
        assert got == exp, (w, h, fmt, next(i for i in range(len(got)) if got[i] != exp[i]))


def png_pixels(png: bytes):
    assert png[:8] == b"\x89PNG\r\n\x1a\n"
    pos, idat = 8, b""
    while pos < len(png):
        n, typ = struct.unpack(">I4s", png[pos:pos + 8])
        data = png[pos + 8:pos + 8 + n]
        assert zlib.crc32(png[pos + 4:pos + 8 + n]) == struct.unpack(">I", png[pos + 8 + n:pos + 12 + n])[0], typ
        if typ == b"IHDR":
            w, h = struct.unpack(">II", data[:8])
        elif typ == b"IDAT":
            idat += data
        pos += 12 + n
    raw = zlib.decompress(idat)  # checks the Adler-32 too
    sb = 3 * w + 1
    assert len(raw) == h * sb and all(raw[y * sb] == 0 for y in range(h))
    return w, h, b"".join(raw[y * sb + 1:(y + 1) * sb] for y in range(h))


def test_png_is_valid_and_matches_ppm(vp8g):
    """Independent check with zlib: chunk CRCs, zlib stream + Adler-32, and the pixels equal the
    PPM payload of the same image."""
    w, h = 1001, 77
    i420 = random_i420(w, h, 5)
    pw, ph, px = png_pixels(vp8g.gpu_encode(i420, w, h, "png"))
    ppm = vp8g.gpu_encode(i420, w, h, "ppm")
    hdr = b"P6\n%d %d\n255\n" % (w, h)
    assert (pw, ph) == (w, h) and ppm.startswith(hdr) and ppm[len(hdr):] == px


@pytest.mark.parametrize("fmt", ["rgb", "ppm", "png"])
def test_device_batch_mixed_sizes(vp8g, fmt):
    """vp8g_encode_batch_device: many images of different sizes in one launch (tasks of several
    images interleave across workgroups), device-resident planes, packed outputs."""
    import torch
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(11)
    sizes = [(int(rng.integers(1, 900)), int(rng.integers(1, 300))) for _ in range(40)] + [(3840, 2160), (1, 1)]
    planes, offs, o = [], [], 0
    for i, (w, h) in enumerate(sizes):
        b = random_i420(w, h, 100 + i)
        cw, ch = (w + 1) // 2, (h + 1) // 2
        offs.append((o, o + w * h, o + w * h + cw * ch))
        planes.append(b)
        o += len(b)
    src = torch.from_numpy(np.frombuffer(b"".join(planes), dtype=np.uint8).copy()).to(dev)
    descs, outs, total, spans = vp8g.make_enc_descs(sizes, fmt, offs)
    lib = vp8g.gpu_lib()
    d_descs = torch.frombuffer(bytearray(bytes(descs)), dtype=torch.uint8).to(dev)
    out = torch.full((total + 16,), 0xEE, dtype=torch.uint8, device=dev)
    work = torch.empty(lib.vp8g_encode_workspace_size(spans), dtype=torch.uint8, device=dev)
    stream = torch.cuda.current_stream(dev)
    assert lib.vp8g_encode_batch_device(descs, C.c_void_p(d_descs.data_ptr()), len(sizes), C.c_void_p(src.data_ptr()),
                                        C.c_void_p(out.data_ptr()), C.c_void_p(work.data_ptr()),
                                        C.c_void_p(stream.cuda_stream)) == 0
    host = out.cpu().numpy().tobytes()
    for i, (w, h) in enumerate(sizes):
        got = host[outs[i]:outs[i] + descs[i].file_len]
        if fmt == "rgb":
            ppm = vp8g.oracle_encode(planes[i], w, h, "ppm")
            exp = ppm[len(b"P6\n%d %d\n255\n" % (w, h)):]
        else:
            exp = vp8g.oracle_encode(planes[i], w, h, fmt)
        assert got == exp, (i, w, h, fmt)


def test_writer_errors(vp8g):
    lib = C.CDLL(str(vp8g.LIB_DIR / "libvp8g.so"), use_errno=True)
    lib.yuv420_write_png_fd.argtypes = [C.c_int, C.POINTER(vp8g.Yuv420Image)]
    lib.yuv420_write_ppm_fd.argtypes = [C.c_int, C.POINTER(vp8g.Yuv420Image)]
    for fn in (lib.yuv420_write_ppm_fd, lib.yuv420_write_png_fd):
        C.set_errno(0)
        assert fn(1, None) == -1 and C.get_errno() == 22
        img = vp8g.Yuv420Image()
        C.set_errno(0)
        assert fn(-1, C.byref(img)) == -1 and C.get_errno() == 22


@pytest.mark.parametrize("rel", ["big/fhd_normal_sharp5.webp", "webp/blockcheck2_16x16_000_000_000_255_255_255_q010.webp",
                                 "commons/penguin-q40.webp", "big/uhd_d_normal_q90.webp"])
@pytest.mark.parametrize("flag", ["-ppm", "-png"])
def test_cli_rgb_end_to_end(manifest, tmp_path, rel, flag):
    """`decoder -ppm/-png in out` (reference src/main.c:706-844; gate scripts/m8_compare_ppm_with_dwebp.sh
    compares -ppm files with dwebp's byte for byte)."""
    out = tmp_path / ("o" + flag[1:])
    r = subprocess.run([str(ROOT / "webp-decoder_amd/bin/decoder"), flag, str(FIXTURES / rel), str(out)],
                       capture_output=True, timeout=300)
    assert r.returncode == 0, r.stderr
    assert sha(out.read_bytes()) == manifest["files"][rel][flag[1:] + "_sha256"]
