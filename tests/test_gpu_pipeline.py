"""GPU tests (MI355X) of the end-to-end batch path vp8g_decode_webp_batch (.webp bytes -> I420):
threaded host m05 into the packed wire format, chunked upload, device expansion, the fused
recon(+LF) kernel, D2H (webp-decoder_amd/csrc/vp8g_pipeline.hip).

Bar: bit-exact against the reference decoder's `-yuv` / `-yuvf` output (sha256 in
tests/golden/manifest.json) for every fixture, in one call, whatever the thread count and chunking.
"""
import hashlib

import pytest

from conftest import FIXTURES, ROOT

pytestmark = pytest.mark.gpu


def sha(b):
    return hashlib.sha256(b).hexdigest()


@pytest.mark.parametrize("filtered,key", [(True, "yuvf_sha256"), (False, "yuv_sha256")])
def test_corpus_one_call(vp8g, manifest, filtered, key):
    rels = sorted(manifest["files"])
    outs, st = vp8g.gpu_decode_webp_batch([(FIXTURES / r).read_bytes() for r in rels], filtered, 16)
    assert st == [0] * len(rels)
    bad = [r for r, o in zip(rels, outs) if sha(o) != manifest["files"][r][key]]
    assert not bad, f"{len(bad)} mismatches, e.g. {bad[:8]}"


def test_thread_counts_and_chunking(vp8g, manifest):
    """Many 4K frames (several chunks, the two device slots alternate) with 1 and 16 threads."""
    rels = ["big/uhd_a_normal_seg4.webp", "big/uhd_b_simple_sharp3.webp", "big/uhd_c_normal_sharp6_seg1.webp",
            "big/k128_normal.webp", "big/fhd_normal_sharp5.webp"]
    files = [(FIXTURES / r).read_bytes() for r in rels]
    seq = [i % len(rels) for i in range(150)]
    for threads in (16, 1):
        use = seq if threads == 16 else seq[:12]
        outs, st = vp8g.gpu_decode_webp_batch([files[i] for i in use], True, threads)
        assert st == [0] * len(use)
        for i, o in zip(use, outs):
            assert sha(o) == manifest["files"][rels[i]]["yuvf_sha256"], (threads, rels[i])


def test_failed_frames_are_isolated(vp8g, manifest):
    good = ["webp/blockcheck2_16x16_000_000_000_255_255_255_q010.webp", "commons/penguin-q20.webp"]
    bad = [(ROOT / "tests" / "fixtures_err" / n).read_bytes() for n in ("empty_riff.webp", "truncated.webp")]
    files = [(FIXTURES / good[0]).read_bytes(), bad[0], b"", (FIXTURES / good[1]).read_bytes(), bad[1]]
    outs, st = vp8g.gpu_decode_webp_batch(files, True, 4)
    assert st[0] == 0 and st[3] == 0 and all(s != 0 for s in (st[1], st[2], st[4]))
    assert outs[1] is None and outs[2] is None and outs[4] is None
    assert sha(outs[0]) == manifest["files"][good[0]]["yuvf_sha256"]
    assert sha(outs[3]) == manifest["files"][good[1]]["yuvf_sha256"]
