"""multi-partition token streams (RFC 6386 9.5; the reference rejects them,
vp8_tokens.c:357-360, and its corpus holds none -- parity unpinned against the reference).

Fixtures are generated from the corpus by re-encoding each frame's decisions with its tokens
spread over 2 / 4 / 8 partitions (tests/multipart.py, oracle/vp8_repartition.c), so the expected
result is the original frame's: same m05 output, same pixels (whose sha256 the reference
decoder produced, tests/golden/manifest.json).  The generator itself is pinned by the 1-partition
re-encode reproducing the original m05 arrays exactly."""
import ctypes as C

import numpy as np
import pytest

from conftest import FIXTURES
from multipart import repartition

SIDE = ("ymode", "uv_mode", "segment_id", "has_coeff", "bmode")


def dense(vp8g, data):
    kf, df, st = vp8g.Vp8KeyFrameHeader(), vp8g.Vp8DecodedFrame(), C.c_int(0)
    buf = (C.c_uint8 * len(data)).from_buffer_copy(data)
    rc = vp8g.host_lib().vp8f_decode_memory(buf, len(data), C.byref(kf), C.byref(df), C.byref(st))
    if rc != 0:
        return None
    f = vp8g.Frame(kf, df)
    out = {k: f.array(k).copy() for k, _, _ in vp8g.FRAME_ARRAYS}
    f.free()
    return out


def test_generator_one_partition_round_trip(vp8g, manifest):
    for rel in sorted(manifest["files"])[::6]:
        data = (FIXTURES / rel).read_bytes()
        a, b = dense(vp8g, data), dense(vp8g, repartition(data, 0))
        assert all(np.array_equal(a[k], b[k]) for k in a), rel


@pytest.mark.parametrize("log2k", [1, 2, 3])
def test_host_multi_partition_equals_original(vp8g, manifest, log2k):
    for rel in sorted(manifest["files"])[::5]:
        data = (FIXTURES / rel).read_bytes()
        m = repartition(data, log2k)
        assert dense(vp8g, m) is None  # the reference-equivalent front end: ENOTSUP
        with pytest.raises(ValueError):
            vp8g.PackedFrame(m)  # opt-in only
        p0, p1 = vp8g.PackedFrame(data), vp8g.PackedFrame(m, multi_partition=True)
        assert np.array_equal(p0.masks(), p1.masks()) and np.array_equal(p0.values(), p1.values()), rel
        assert all(np.array_equal(p0.side(k), p1.side(k)) for k in SIDE), rel


def test_partition_table_rejects_overruns(vp8g, manifest):
    data = (FIXTURES / sorted(manifest["files"])[3]).read_bytes()
    m = bytearray(repartition(data, 2))
    tag = m[20] | m[21] << 8 | m[22] << 16
    fpl = tag >> 5
    m[20 + 10 + fpl:20 + 10 + fpl + 3] = b"\xff\xff\xff"  # first partition size past the end
    with pytest.raises(ValueError):
        vp8g.PackedFrame(bytes(m), multi_partition=True)


def test_token_header_partition_table(vp8g, manifest):
    """The device job of a multi-partition frame lists the partitions (opt-in), contiguous after
    the size table, the last one ending at the payload's end."""
    data = (FIXTURES / sorted(manifest["files"])[7]).read_bytes()
    for log2k in (1, 2, 3):
        m = repartition(data, log2k)
        with pytest.raises(ValueError):
            vp8g.token_header(m)
        kf, hdr, tf, off, size = vp8g.token_header(m, multi_partition=True)
        k = 1 << log2k
        assert tf.nparts == k
        assert tf.part_off[0] == 10 + kf.first_partition_len + 3 * (k - 1) == tf.tok_off
        assert all(tf.part_off[p + 1] == tf.part_end[p] for p in range(k - 1)) and tf.part_end[k - 1] == size


def test_m05_launcher_validates_jobs(vp8g, manifest):
    """vp8g_m05_batch_device checks every job on the host before anything reaches the device
    (inconsistent jobs -> EINVAL, no launch): partition counts, partition order, bool state,
    dimensions, alignment, and the required status word.  Runs without a GPU."""
    import ctypes as C
    lib = vp8g.gpu_lib()
    data = repartition((FIXTURES / sorted(manifest["files"])[5]).read_bytes(), 2)
    _, _, tf, _, _ = vp8g.token_header(data, multi_partition=True)
    status = C.c_uint32(0)
    arr = vp8g.Vp8gBatchArrays(**{k: 16 for k in ("coeff_y", "coeff_u", "coeff_v", "coeff_y2", "ymode", "uv_mode",
                                                  "segment_id", "has_coeff", "bmode")},
                               src=None, status=C.addressof(status))

    def call(job, arrays=arr):
        jobs = (vp8g.Vp8gTokFrame * 1)(job)
        C.set_errno(0)
        return lib.vp8g_m05_batch_device(jobs, 16, 1, 16, C.byref(arrays), None)

    def bad(**fields):
        j = vp8g.Vp8gTokFrame.from_buffer_copy(bytes(tf))
        for k, v in fields.items():
            if isinstance(v, tuple):
                getattr(j, k)[v[0]] = v[1]
            else:
                setattr(j, k, v)
        return j

    for job in (bad(nparts=3), bad(nparts=16), bad(mb_cols=0), bad(mb_rows=2000), bad(data=2), bad(b_range=300),
                bad(b_bits=-1), bad(b_next=tf.p0_end + 1), bad(part_off=(1, tf.part_end[0] - 1)),
                bad(part_off=(0, tf.p0_end - 1))):
        assert call(job) == -1 and C.get_errno() == 22
    no_status = vp8g.Vp8gBatchArrays.from_buffer_copy(bytes(arr))
    no_status.status = None
    assert call(tf, no_status) == -1 and C.get_errno() == 22
