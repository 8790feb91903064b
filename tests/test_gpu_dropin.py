"""GPU: the reference's OWN CLI re-linked against the drop-in.

oracle/_ref/decoder_vp8g   = the reference's src/main.c + m01-m05 (+ m04, m08, m09) compiled from the
                             reference sources (oracle/Makefile) with NO vp8_recon.c / vp8_loopfilter.c,
                             linked against libvp8g.so: its -yuv / -yuvf / -ppm / -png calls
                             (src/main.c:591, :665, :742, :811) run our HIP path;
oracle/_ref/decoder_vp8g_rgb = the same without m08/m09: -ppm / -png also run libvp8g's device writers.
oracle/_ref/decoder_ultra_vp8g[_rgb] = the reference's src/main_ultra.c (PNG-only CLI) re-linked the same
                             way: its one call (src/main_ultra.c:43) runs our HIP path.
-diff_mb (src/main.c:881, unfiltered recon vs an oracle I420, per-segment SAD report) is compared line
for line with the reference's own decoder (oracle/_ref/decoder) given the same oracle file.
Outputs are byte-compared with the reference's own (tests/golden/manifest.json), like its gates
(scripts/m6_compare_yuv_with_dwebp.sh:69, m7_compare_yuv_filtered_with_oracle.sh:66).  The binaries are
built here in the container (they need the reference sources) and travel to the GPU box prebuilt.
"""
import hashlib
import subprocess

import pytest

from conftest import FIXTURES, ROOT

pytestmark = pytest.mark.gpu

BIN = ROOT / "oracle" / "_ref"
SAMPLE = ["big/k128_normal.webp", "big/fhd_normal_sharp5.webp", "big/fhd_simple_sharp3.webp",
          "big/uhd_b_simple_sharp3.webp", "big/odd_1917x1083_normal.webp", "commons/penguin-q40.webp",
          "webp/blockcheck2_16x16_000_000_000_255_255_255_q010.webp"]


def sample(manifest):
    rels = sorted(manifest["files"])
    return SAMPLE + rels[::37]


@pytest.mark.parametrize("binary", ["decoder_vp8g", "decoder_vp8g_rgb"])
@pytest.mark.parametrize("flag,key", [("-yuv", "yuv_sha256"), ("-yuvf", "yuvf_sha256"), ("-ppm", "ppm_sha256"),
                                      ("-png", "png_sha256")])
def test_reference_cli_relinked(manifest, tmp_path, binary, flag, key):
    exe = BIN / binary
    if not exe.exists():
        pytest.skip(f"{exe} not built (needs the reference sources at build time)")
    bad = []
    for rel in sample(manifest):
        out = tmp_path / "o.bin"
        r = subprocess.run([str(exe), flag, str(FIXTURES / rel), str(out)], capture_output=True, timeout=300)
        if r.returncode != 0 or hashlib.sha256(out.read_bytes()).hexdigest() != manifest["files"][rel][key]:
            bad.append((rel, r.returncode, r.stderr[-200:]))
    assert not bad, bad[:4]


@pytest.mark.parametrize("binary", ["decoder_vp8g", "decoder_vp8g_rgb"])
def test_reference_cli_diff_mb(manifest, tmp_path, binary):
    """`decoder -diff_mb in.webp oracle.i420` (src/main.c:846-1017): the relinked binary's report
    equals the reference's.  The oracle file is the reference's -yuvf output, so the SADs are the
    loop filter's per-segment footprint (non-zero), and a truncated copy exercises the size check."""
    exe, ref = BIN / binary, BIN / "decoder"
    if not exe.exists() or not ref.exists():
        pytest.skip("not built (needs the reference sources at build time)")
    bad = []
    for rel in sample(manifest):
        orc = tmp_path / "oracle.i420"
        r = subprocess.run([str(ref), "-yuvf", str(FIXTURES / rel), str(orc)], capture_output=True, timeout=300)
        assert r.returncode == 0, rel
        for trunc in (False, True):
            if trunc:
                orc.write_bytes(orc.read_bytes()[:-1])
            a = subprocess.run([str(exe), "-diff_mb", str(FIXTURES / rel), str(orc)], capture_output=True, timeout=300)
            b = subprocess.run([str(ref), "-diff_mb", str(FIXTURES / rel), str(orc)], capture_output=True, timeout=300)
            if (a.returncode, a.stdout, a.stderr) != (b.returncode, b.stdout, b.stderr):
                bad.append((rel, trunc, a.returncode, b.returncode, a.stdout[-200:], b.stdout[-200:]))
            elif not trunc:
                assert b"Total SAD" in a.stdout
    assert not bad, bad[:3]


@pytest.mark.parametrize("binary", ["decoder_ultra_vp8g", "decoder_ultra_vp8g_rgb"])
def test_reference_ultra_cli_relinked(manifest, tmp_path, binary):
    """src/main_ultra.c (decoder_nolibc_ultra's source, PNG only, exit 0 / 1 / 2) re-linked against
    libvp8g.so: its PNGs equal the reference's (manifest png_sha256)."""
    exe = BIN / binary
    if not exe.exists():
        pytest.skip(f"{exe} not built (needs the reference sources at build time)")
    bad = []
    for rel in sample(manifest):
        out = tmp_path / "o.png"
        r = subprocess.run([str(exe), str(FIXTURES / rel), str(out)], capture_output=True, timeout=300)
        if r.returncode != 0 or hashlib.sha256(out.read_bytes()).hexdigest() != manifest["files"][rel]["png_sha256"]:
            bad.append((rel, r.returncode))
    assert not bad, bad[:4]
    assert subprocess.run([str(exe), "only-one-arg"], capture_output=True).returncode == 2
    assert subprocess.run([str(exe), str(tmp_path / "missing.webp"), str(tmp_path / "x.png")],
                          capture_output=True).returncode == 1


def test_relinked_binaries_do_not_contain_reference_recon():
    """The m06/m07 symbols must come from libvp8g.so (undefined in the executable)."""
    for binary, syms in (("decoder_vp8g", ("vp8_reconstruct_keyframe_yuv", "vp8_reconstruct_keyframe_yuv_filtered")),
                         ("decoder_vp8g_rgb", ("vp8_reconstruct_keyframe_yuv", "vp8_reconstruct_keyframe_yuv_filtered")),
                         ("decoder_ultra_vp8g", ("vp8_reconstruct_keyframe_yuv_filtered",)),
                         ("decoder_ultra_vp8g_rgb", ("vp8_reconstruct_keyframe_yuv_filtered", "yuv420_write_png_fd"))):
        exe = BIN / binary
        if not exe.exists():
            pytest.skip("not built")
        nm = subprocess.run(["nm", "-D", "--undefined-only", str(exe)], capture_output=True, text=True).stdout
        for sym in syms:
            assert f" U {sym}\n" in nm + "\n", (binary, sym)
