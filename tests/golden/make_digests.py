#!/usr/bin/env python3
"""Generate tests/golden/digests.json and tests/golden/multipart.json (run HERE, where the
reference and libwebp exist; the GPU box reads only the JSON).

digests.json    the device digest (include/vp8g.h vp8g_frame_digests; numpy restatement
                vp8g.digest64) of the reference decoder's own -yuv / -yuvf I420
                (oracle/_ref/libref.so = the reference's m01-m07 compiled in place) for
                  * the bench fixtures (4 x 3840x2160, 4 x 1920x1080), and
                  * the bench's synthetic 4K batch: vp8_synth.c profile 0, seed 0x5EED ^ i for the
                    global frame index i in [0, 4096) (BASELINE configs 4 and 5: 512 frames per GPU
                    on up to 8 GPUs), -yuvf only.
                The bench checks every frame of every rank against these.
multipart.json  2/4/8-partition token streams encoded here by libwebp 1.2.2 (tools/make_big_fixtures.c,
                tests/fixtures_mp/): the reference rejects them (src/m05_tokens/vp8_tokens.c:357-360,
                ENOTSUP), so their expected I420 is libwebp's own decode (oracle/libwebp_probe.c, the
                library behind the reference's dwebp gates): sha256 + digest of -yuv / -yuvf.
"""
import hashlib
import json
import multiprocessing as mp
import pathlib
import subprocess
import sys
import tempfile

ROOT = pathlib.Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT / "webp-decoder_amd"))
import vp8g  # noqa: E402

FIX = ROOT / "tests" / "fixtures"
FIX_MP = ROOT / "tests" / "fixtures_mp"
PROBE = ROOT / "oracle" / "_ref" / "libwebp_probe"
BENCH_FIXTURES = ["big/uhd_a_normal_seg4.webp", "big/uhd_b_simple_sharp3.webp", "big/uhd_c_normal_sharp6_seg1.webp",
                  "big/uhd_d_normal_q90.webp", "big/fhd_normal_sharp5.webp", "big/fhd_simple_sharp3.webp",
                  "big/fhd_c_normal_q85_seg4.webp", "big/fhd_d_normal_sharp2_seg1.webp"]
SYNTH_W, SYNTH_H, SYNTH_SEED, SYNTH_PROFILE, SYNTH_FRAMES = 3840, 2160, 0x5EED, 0, 4096


def hx(d: int) -> str:
    return "0x%016x" % d


def ref_i420(path: pathlib.Path, filtered: int) -> bytes:
    import numpy as np
    lib = vp8g.ref_lib()
    n = lib.ref_decode_i420(str(path).encode(), None, 0, filtered)
    assert n > 0, (path, n)
    buf = np.empty(n, dtype=np.uint8)
    assert lib.ref_decode_i420(str(path).encode(), buf.ctypes.data, n, filtered) == n
    return buf.tobytes()


def synth_digest(i: int) -> str:
    f = vp8g.synth_frame(SYNTH_W, SYNTH_H, SYNTH_SEED ^ i, SYNTH_PROFILE)
    d = vp8g.digest64(vp8g.ref_reconstruct(f, True))
    f.free()
    return hx(d)


def libwebp_i420(path: pathlib.Path, filtered: int) -> bytes:
    with tempfile.NamedTemporaryFile(suffix=".i420") as t:
        args = [str(PROBE)] + ([] if filtered else ["-nofilter"]) + [str(path), t.name]
        subprocess.run(args, check=True, capture_output=True)
        return pathlib.Path(t.name).read_bytes()


def main():
    out = {"generator": "tests/golden/make_digests.py", "digest": "include/vp8g.h vp8g_frame_digests (vp8g.digest64)",
           "reference": "oracle/_ref/libref.so (reference m01-m07)", "fixtures": {}}
    for rel in BENCH_FIXTURES:
        p = FIX / rel
        out["fixtures"][rel] = {"yuv": hx(vp8g.digest64(ref_i420(p, 0))), "yuvf": hx(vp8g.digest64(ref_i420(p, 1)))}
    with mp.Pool(8) as pool:
        dig = pool.map(synth_digest, range(SYNTH_FRAMES), chunksize=16)
    out["synth_uhd"] = {"width": SYNTH_W, "height": SYNTH_H, "profile": SYNTH_PROFILE, "seed": "0x5EED ^ i",
                        "frames": SYNTH_FRAMES, "yuvf": dig}
    (ROOT / "tests" / "golden" / "digests.json").write_text(json.dumps(out, indent=0) + "\n")
    print("digests:", len(out["fixtures"]), "fixtures,", len(dig), "synthetic frames")

    mpj = {"generator": "tests/golden/make_digests.py", "oracle": "libwebp 1.2.2 (oracle/libwebp_probe.c)",
           "encoder": "tools/make_big_fixtures.c (libwebp 1.2.2, WebPConfig.partitions, low_memory)", "files": {}}
    for p in sorted(FIX_MP.glob("*.webp")):
        kf, hdr, tf, off, size = vp8g.token_header(p.read_bytes(), multi_partition=True)
        ent = {"width": int(kf.width), "height": int(kf.height), "partitions": int(tf.nparts)}
        for filt, key in ((0, "yuv"), (1, "yuvf")):
            b = libwebp_i420(p, filt)
            ent[key + "_sha256"] = hashlib.sha256(b).hexdigest()
            ent[key + "_digest"] = hx(vp8g.digest64(b))
        mpj["files"][p.name] = ent
    (ROOT / "tests" / "golden" / "multipart.json").write_text(json.dumps(mpj, indent=1, sort_keys=True) + "\n")
    print("multipart:", len(mpj["files"]), "files")


if __name__ == "__main__":
    main()
