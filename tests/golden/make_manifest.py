#!/usr/bin/env python3
"""Generate the golden manifests under tests/golden/ (run HERE, where /root/reference exists).

manifest.json   for every fixture under tests/fixtures/**.webp: width, height, the reference
                front end's FNV-1a coefficient hash, and sha256 of the reference decoder's
                `-yuv` and `-yuvf` output (oracle/_ref/libref.so = the reference's own m01-m07
                compiled in place by oracle/Makefile).  Each output is also cross-checked against
                libwebp 1.2.2 (oracle/_ref/libwebp_probe, the library behind the reference's
                `dwebp` oracle gates scripts/m6_*.sh, scripts/m7_*.sh); the result is recorded.
                Also sha256 of the reference decoder's `-ppm` and `-png` files (m08/m09, the
                `decoder` binary compiled from the reference by oracle/Makefile), cross-checked
                against libwebp's RGB (the `dwebp -ppm` payload) and, for the 90 files of the
                reference's images/webp, against the pixels of its dwebp PNG goldens
                (images/png-out/*.png, decoded here with zlib).
synth_kat.json  seeded synthetic Vp8DecodedFrames (webp-decoder_amd/host/vp8_synth.c spec) ->
                sha256 of the reference m06 / m06+m07 output.

These are data (inputs are the fixture files / the generator spec, outputs are hashes); the GPU
box needs only them, never the reference.
"""
import hashlib
import json
import pathlib
import subprocess
import sys
import tempfile

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT / "webp-decoder_amd"))
import vp8g  # noqa: E402

FIX = ROOT / "tests" / "fixtures"
PROBE = ROOT / "oracle" / "_ref" / "libwebp_probe"

# (width, height, seed, profile): sizes straddle MB boundaries; profiles see vp8_synth.c
SYNTH_CASES = [
    (1, 1, 1, 0), (1, 1, 2, 1), (16, 16, 3, 0), (17, 17, 4, 1), (31, 33, 5, 2), (64, 48, 6, 0),
    (129, 77, 7, 1), (200, 150, 8, 2), (333, 97, 9, 0), (16, 400, 10, 1), (400, 16, 11, 2),
    (640, 480, 12, 0), (641, 481, 13, 1), (1920, 1080, 14, 0), (1920, 1080, 15, 1), (1917, 1083, 16, 2),
    (3840, 2160, 0x5EED, 0),
]


def sha(b: bytes) -> str:
    return hashlib.sha256(b).hexdigest()


def ref_i420(path: pathlib.Path, filtered: int) -> bytes:
    lib = vp8g.ref_lib()
    n = lib.ref_decode_i420(str(path).encode(), None, 0, filtered)
    assert n > 0, (path, n)
    buf = np.empty(n, dtype=np.uint8)
    assert lib.ref_decode_i420(str(path).encode(), buf.ctypes.data, n, filtered) == n
    return buf.tobytes()


def libwebp_i420(path: pathlib.Path, filtered: int) -> bytes | None:
    if not PROBE.exists():
        return None
    with tempfile.NamedTemporaryFile(suffix=".i420") as t:
        args = [str(PROBE)] + ([] if filtered else ["-nofilter"]) + [str(path), t.name]
        if subprocess.run(args, capture_output=True).returncode != 0:
            return None
        return pathlib.Path(t.name).read_bytes()


REF_DECODER = ROOT / "oracle" / "_ref" / "decoder"
PNG_OUT = pathlib.Path("/root/reference/images/png-out")


def ref_file(path: pathlib.Path, fmt: str) -> bytes:
    with tempfile.NamedTemporaryFile(suffix="." + fmt) as t:
        r = subprocess.run([str(REF_DECODER), "-" + fmt, str(path), t.name], capture_output=True)
        assert r.returncode == 0, (path, fmt, r.stderr)
        return pathlib.Path(t.name).read_bytes()


def libwebp_rgb(path: pathlib.Path) -> bytes | None:
    if not PROBE.exists():
        return None
    with tempfile.NamedTemporaryFile(suffix=".rgb") as t:
        if subprocess.run([str(PROBE), "-rgb", str(path), t.name], capture_output=True).returncode != 0:
            return None
        return pathlib.Path(t.name).read_bytes()


def png_pixels(png: bytes) -> tuple[int, int, bytes]:
    """RGB24 rows of an 8-bit RGB, non-interlaced PNG (any filter types), via zlib."""
    import struct
    import zlib
    assert png[:8] == b"\x89PNG\r\n\x1a\n"
    pos, idat, w, h = 8, b"", 0, 0
    while pos < len(png):
        n, typ = struct.unpack(">I4s", png[pos:pos + 8])
        data = png[pos + 8:pos + 8 + n]
        if typ == b"IHDR":
            w, h, depth, ctype = struct.unpack(">IIBB", data[:10])
            assert depth == 8 and ctype == 2
        elif typ == b"IDAT":
            idat += data
        pos += 12 + n
    raw = zlib.decompress(idat)
    sb, out, prev = 3 * w + 1, bytearray(), bytearray(3 * w)
    for y in range(h):
        ft, line = raw[y * sb], bytearray(raw[y * sb + 1:(y + 1) * sb])
        for i in range(3 * w):
            a = line[i - 3] if i >= 3 else 0
            b = prev[i]
            c = prev[i - 3] if i >= 3 else 0
            if ft == 1:
                line[i] = (line[i] + a) & 255
            elif ft == 2:
                line[i] = (line[i] + b) & 255
            elif ft == 3:
                line[i] = (line[i] + ((a + b) >> 1)) & 255
            elif ft == 4:
                p = a + b - c
                pa, pb, pc = abs(p - a), abs(p - b), abs(p - c)
                line[i] = (line[i] + (a if pa <= pb and pa <= pc else (b if pb <= pc else c))) & 255
        out += line
        prev = line
    return w, h, bytes(out)


def main():
    files = sorted(FIX.rglob("*.webp"))
    out = {"generator": "tests/golden/make_manifest.py", "reference": "oracle/_ref/libref.so (reference m01-m07)",
           "libwebp": "1.2.2 (system library, dwebp-equivalent probe)", "files": {}}
    agree = {"yuv": 0, "yuvf": 0, "rgb": 0, "png_out": 0}
    n_gold = 0
    for p in files:
        rel = str(p.relative_to(FIX))
        f = vp8g.decode_file(p)
        ent = {"width": f.width, "height": f.height, "mb_cols": int(f.frame.mb_cols), "mb_rows": int(f.frame.mb_rows),
               "coeff_hash": "0x%016x" % vp8g.ref_lib().ref_coeff_hash(str(p).encode()),
               "lf_simple": int(f.frame.lf_use_simple), "lf_level": int(f.frame.lf_level),
               "lf_sharpness": int(f.frame.lf_sharpness), "segmentation": int(f.frame.segmentation_enabled)}
        for filt, key in ((0, "yuv"), (1, "yuvf")):
            r = ref_i420(p, filt)
            ent[key + "_sha256"] = sha(r)
            w = libwebp_i420(p, filt)
            ent["libwebp_" + key] = None if w is None else (w == r)
            agree[key] += int(w == r)
        ppm, png = ref_file(p, "ppm"), ref_file(p, "png")
        ent["ppm_sha256"], ent["png_sha256"] = sha(ppm), sha(png)
        hdr = b"P6\n%d %d\n255\n" % (f.width, f.height)
        rgb = ppm[len(hdr):]
        lw = libwebp_rgb(p)
        ent["libwebp_rgb"] = None if lw is None else (ppm.startswith(hdr) and lw == rgb)
        agree["rgb"] += int(bool(ent["libwebp_rgb"]))
        gold = PNG_OUT / (p.stem + ".png")
        if rel.startswith("webp/") and gold.exists():
            gw, gh, gpx = png_pixels(gold.read_bytes())
            ent["dwebp_png_out"] = (gw, gh) == (f.width, f.height) and gpx == rgb
            agree["png_out"] += int(ent["dwebp_png_out"])
            n_gold += 1
        out["files"][rel] = ent
        f.free()
    out["libwebp_agreement"] = {k: f"{v}/{n_gold if k == 'png_out' else len(files)}" for k, v in agree.items()}
    (ROOT / "tests" / "golden" / "manifest.json").write_text(json.dumps(out, indent=1, sort_keys=True) + "\n")
    print("manifest:", len(files), "files; libwebp agreement", out["libwebp_agreement"])

    kat = {"generator": "tests/golden/make_manifest.py", "spec": "webp-decoder_amd/host/vp8_synth.c", "cases": []}
    for (w, h, seed, prof) in SYNTH_CASES:
        f = vp8g.synth_frame(w, h, seed, prof)
        kat["cases"].append({"width": w, "height": h, "seed": seed, "profile": prof,
                             "yuv_sha256": sha(vp8g.ref_reconstruct(f, False)),
                             "yuvf_sha256": sha(vp8g.ref_reconstruct(f, True))})
        f.free()
    (ROOT / "tests" / "golden" / "synth_kat.json").write_text(json.dumps(kat, indent=1) + "\n")
    print("synth KAT:", len(SYNTH_CASES), "cases")


if __name__ == "__main__":
    main()
