#!/usr/bin/env python3
"""Generate the golden manifests under tests/golden/ (run HERE, where /root/reference exists).

manifest.json   for every fixture under tests/fixtures/**.webp: width, height, the reference
                front end's FNV-1a coefficient hash, and sha256 of the reference decoder's
                `-yuv` and `-yuvf` output (oracle/_ref/libref.so = the reference's own m01-m07
                compiled in place by oracle/Makefile).  Each output is also cross-checked against
                libwebp 1.2.2 (oracle/_ref/libwebp_probe, the library behind the reference's
                `dwebp` oracle gates scripts/m6_*.sh, scripts/m7_*.sh); the result is recorded.
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


def main():
    files = sorted(FIX.rglob("*.webp"))
    out = {"generator": "tests/golden/make_manifest.py", "reference": "oracle/_ref/libref.so (reference m01-m07)",
           "libwebp": "1.2.2 (system library, dwebp-equivalent probe)", "files": {}}
    agree = {"yuv": 0, "yuvf": 0}
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
        out["files"][rel] = ent
        f.free()
    out["libwebp_agreement"] = {k: f"{v}/{len(files)}" for k, v in agree.items()}
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
