"""Split mode (small batches: one frame worked on by several workgroups that hand MB-row-pair
context to each other through a device-memory mailbox) vs the oracle, at forced split factors.

VP8G_SPLIT / VP8G_WAVES are read by the shim on every call (webp-decoder_amd/csrc/vp8g_shim.hip
run_locked); VP8G_SPLIT=1 forces the one-workgroup-per-frame path.
"""
import os

import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture
def env():
    saved = {k: os.environ.get(k) for k in ("VP8G_SPLIT", "VP8G_WAVES")}
    yield os.environ
    for k, v in saved.items():
        if v is None:
            os.environ.pop(k, None)
        else:
            os.environ[k] = v


@pytest.mark.parametrize("split,waves", [(1, 0), (1, 16), (2, 8), (3, 8), (8, 8), (5, 16)])
def test_split_factors_vs_oracle(vp8g, env, split, waves):
    env["VP8G_SPLIT"] = str(split)
    if waves:
        env["VP8G_WAVES"] = str(waves)
    else:
        env.pop("VP8G_WAVES", None)
    cases = [(1920, 1080, 11, 1), (1917, 1083, 12, 2), (333, 470, 13, 0), (16, 900, 14, 1), (1280, 720, 15, 0),
             (64, 64, 16, 2)]
    frames = [vp8g.synth_frame(w, h, s, p) for w, h, s, p in cases]
    for filtered in (False, True):
        outs = vp8g.gpu_reconstruct_batch(frames, filtered)
        for f, o in zip(frames, outs):
            assert o == vp8g.oracle_reconstruct(f, filtered), (f.width, f.height, filtered, split, waves)
        one = vp8g.gpu_reconstruct(frames[0], filtered)
        assert one == outs[0]


def test_split_4k_single_frame_vs_manifest(vp8g, env, manifest):
    """The drop-in single-frame call on a 4K fixture at the default (automatic) split."""
    import hashlib

    from conftest import FIXTURES
    env.pop("VP8G_SPLIT", None)
    env.pop("VP8G_WAVES", None)
    for rel in ("big/uhd_c_normal_sharp6_seg1.webp", "big/uhd_b_simple_sharp3.webp"):
        f = vp8g.decode_file(FIXTURES / rel)
        for filtered, key in ((False, "yuv_sha256"), (True, "yuvf_sha256")):
            assert hashlib.sha256(vp8g.gpu_reconstruct(f, filtered)).hexdigest() == manifest["files"][rel][key]
